# kernel + memory-copy timeline of the flagship with the host-history EvalMonitor vs the device one
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in host device; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_mon_$m -o run --output-format csv -- python3 $R/bench.py --monitor $m --steps 20 --phase-steps 0 > $R/gpurun_out/prof_mon_$m.log 2>&1 || exit 1
  cd $R
  f=$(find gpurun_out/prof_mon_$m -name '*kernel_trace.csv' | head -1)
  python tools/ktrace_gen.py $f --quiet | tail -5
done
