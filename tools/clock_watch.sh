# sample the GPU shader clock / power while a workload runs: tools/clock_watch.sh OUT cmd...
out=$1; shift
"$@" > $out.run.log 2>&1 &
pid=$!
sleep 1
for i in $(seq 1 80); do
  kill -0 $pid 2>/dev/null || break
  { date +%s.%N; /opt/rocm/bin/rocm-smi --showclocks --showpower 2>&1 | grep -E "sclk|Power|fclk|mclk"; } >> $out.clk.txt
  sleep 0.2
done
wait $pid
