set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s4
timeout -k 10 200 python -u scratch8/sim8probe.py pinned > gpurun_out/s4/p.log 2>&1 || { tail -5 gpurun_out/s4/p.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s4/p.log
bash scratch8/s2.sh
