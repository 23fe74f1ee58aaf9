set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s8
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --phase-steps 0 > gpurun_out/s8/$name.log 2>&1 || { echo "$name FAILED"; tail -3 gpurun_out/s8/$name.log; return 0; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/s8/$name.log').read().strip().splitlines()[-1]);e=d['eigh_stats'];print('$name', d['ms_per_step'], e['capped'], e['iters_per_gen'][-10:])"
}
run base A=1
run devkernarg HIP_FORCE_DEV_KERNARG=1
run pktcap1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run pktcap0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run optflush1 AMD_OPT_FLUSH=1
run optflush0 AMD_OPT_FLUSH=0
run sysscope0 ROC_SYSTEM_SCOPE_SIGNAL=0
run hdpwa0 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0
run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64
run batch1024 DEBUG_HIP_GRAPH_BATCH_SIZE=1024
run kcopy0 DEBUG_HIP_KERNARG_COPY_OPT=0
run base2 A=1
