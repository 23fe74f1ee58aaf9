set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
timeout -k 10 200 python -u scratch8/sim8probe.py new1 > gpurun_out/s3/new1.log 2>&1 || { tail -5 gpurun_out/s3/new1.log; exit 1; }
timeout -k 10 200 python -u scratch8/sim8probe.py new2 > gpurun_out/s3/new2.log 2>&1 || { tail -5 gpurun_out/s3/new2.log; exit 1; }
cp evoxmi/_C.so /tmp/_C_new.so && cp scratch8/_C_old.so evoxmi/_C.so
timeout -k 10 200 python -u scratch8/sim8probe.py old1 > gpurun_out/s3/old1.log 2>&1 || { tail -5 gpurun_out/s3/old1.log; exit 1; }
timeout -k 10 200 python -u scratch8/sim8probe.py old2 > gpurun_out/s3/old2.log 2>&1 || { tail -5 gpurun_out/s3/old2.log; exit 1; }
cat gpurun_out/s3/*.log | grep -v amdgpu.ids
