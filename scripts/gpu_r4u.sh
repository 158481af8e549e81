#!/bin/bash
# round-4 GPU call: the default line after encode_batch_host stopped creating a fifth stream
# (4 GiB commit window), plus the host-path GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --cpu-sample 0 > $O/nocpu.json 2> $O/nocpu.err || exit 1
python3 -c "
import json; d=json.load(open('$O/nocpu.json')); x=d['copy_inclusive_encode_commit']; print(x['by_window'], x['stream_writer'], d['copy_inclusive']['value'], d['value'])"
