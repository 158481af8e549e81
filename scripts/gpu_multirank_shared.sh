#!/bin/bash
# the N > 1 bench paths on a one-GPU box: two ranks sharing cuda:0, timings over gloo
# (TEC_BENCH_SHARED_GPU=1); the driver's 8-GPU run uses RCCL, one GPU per rank
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/multirank
mkdir -p $O
export TEC_BENCH_SHARED_GPU=1
timeout -k 10 500 python -u bench.py --gpus 2 --steps 5 --warmup 2 --cpu-sample 0 > $O/default_n2.json 2> $O/default_n2.err && python3 -c "import json; d=json.loads([l for l in open('$O/default_n2.json') if l.startswith('{')][0]); print('default n2', d['n_gpus'], d['world_size'], d['backend'], d['value'], d['roofline']['frac'], d['copy_inclusive']['value'], d['stream_sdk_shape']['value'], d['outputs_verified'] if 'outputs_verified' in d else '')" &&
timeout -k 10 300 python -u bench.py --gpus 2 --mode repair --steps 5 --warmup 2 --cpu-sample 0 > $O/repair_n2.json 2> $O/repair_n2.err && python3 -c "import json; d=json.loads([l for l in open('$O/repair_n2.json') if l.startswith('{')][0]); print('repair n2', d['n_gpus'], d['value'], d['outputs_verified'])" &&
timeout -k 10 300 python -u bench.py --gpus 2 --mode decode --pattern random --steps 5 --warmup 2 --cpu-sample 0 > $O/decode_n2.json 2> $O/decode_n2.err && python3 -c "import json; d=json.loads([l for l in open('$O/decode_n2.json') if l.startswith('{')][0]); print('decode n2', d['n_gpus'], d['value'], d['outputs_verified'])" &&
timeout -k 10 300 python -u bench.py --gpus 2 --mode outer --steps 3 --warmup 1 --cpu-sample 0 > $O/outer_n2.json 2> $O/outer_n2.err && python3 -c "import json; d=json.loads([l for l in open('$O/outer_n2.json') if l.startswith('{')][0]); print('outer n2', d['n_gpus'], d['value'], d['outputs_verified'])" &&
timeout -k 10 600 python -u bench.py --gpus 2 --workload config5 --steps 1 --warmup 1 --cpu-sample 0 > $O/config5_n2.json 2> $O/config5_n2.err && python3 -c "import json; d=json.loads([l for l in open('$O/config5_n2.json') if l.startswith('{')][0]); print('config5 n2', d['n_gpus'], d['objects_per_gpu'] if 'objects_per_gpu' in d else '', d['value'], d['outputs_verified'])"
