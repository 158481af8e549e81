#!/bin/bash
# Time kbench variants scripts/kbench_<name> (quick mode, 1024 objects); name "st" = the stage kernel.
cd $GRAFT_REPO_ROOT
for v in "$@"; do a=""; [ "$v" == st ] && a=s; echo -n "$v: "; timeout -k 5 60 ./scripts/kbench_$v 1024 r q $a | grep full || exit $?; done
