set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s32
run() {  # label env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/s32/$lab.log 2>&1 || { echo "$lab FAILED"; tail -5 gpurun_out/s32/$lab.log; return 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/s32/$lab.log').read().strip().splitlines()[-1])
e=d.get('eigh_stats',{})
print('$lab', d['ms_per_step'], d['config'].get('eigh'), d['config'].get('hipgraph'), {k: e.get(k) for k in ('capped','fallbacks','max_off_rel','mean_refine_iters')})
"
}
run x6 EVOXMI_SBR_CORR_PREC=x6 || exit 1
run x3all EVOXMI_SBR_CORR_PREC=x3all || exit 1
run blas EVOXMI_PLAIN_GEMM=blas || exit 1
run host EVOXMI_SBR_MODE=host || exit 1
run jacobi EVOXMI_EIGH=jacobi || exit 1
run unfused EVOXMI_CMA_FUSED=0 || exit 1
