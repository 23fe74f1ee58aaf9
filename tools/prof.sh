#!/bin/bash
# rocprofv3 kernel stats of an arbitrary python script: tools/prof.sh NAME script.py args...
set -o pipefail
export TMPDIR=/tmp
name=$1; shift
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof_$name
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$name -o run --output-format csv -- python3 "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_$name.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -3 gpurun_out/prof_$name.log
f=$(find gpurun_out/prof_$name -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-250 "$f" | head -${TOPN:-20}
exit $rc
