set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/s5
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s5/kt1 -o kt --output-format csv -- python3 $R/bench.py --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s5/kt1.log 2>&1 || { tail -20 $R/gpurun_out/s5/kt1.log; exit 1; }
for W in 2 8; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/s5/kt$W -o kt --output-format csv -- python3 $R/bench.py --simulate-rank 0 --world $W --steps 40 --warmup 5 --phase-steps 0 > $R/gpurun_out/s5/kt$W.log 2>&1 || { tail -20 $R/gpurun_out/s5/kt$W.log; exit 1; }
done
cd $R
f1=$(find gpurun_out/s5/kt1 -name '*kernel_trace.csv' | head -1)
f2=$(find gpurun_out/s5/kt2 -name '*kernel_trace.csv' | head -1)
f8=$(find gpurun_out/s5/kt8 -name '*kernel_trace.csv' | head -1)
python tools/ktrace_phases.py --gens 20 $f1 $f2 $f8 --labels "1 GPU" "rank 0 of 2 (sim)" "rank 0 of 8 (sim)" > gpurun_out/s5/phases.txt
python tools/ktrace_gen.py $f8 --marker philox_words --show -2 --agg 20 > gpurun_out/s5/kt_gen8.txt
cat gpurun_out/s5/phases.txt
for W in 1 2 8; do tail -1 gpurun_out/s5/kt$W.log | grep -o '"ms_per_step": [0-9.]*\|"projected_ms_with_wire": [0-9.]*\|"schedule_per_gen": "[A-Z]*"' | tr '\n' ' '; echo; done
gzip -f $f1 $f2 $f8
