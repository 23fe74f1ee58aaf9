set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sec
o=gpurun_out/sec
timeout -k 10 200 python tools/bench_mo.py --algo nsga2 > $o/nsga2.json 2>>$o/err || { tail $o/err; exit 1; }
timeout -k 10 200 python tools/bench_mo.py --algo moead > $o/moead_1.json 2>>$o/err || { tail $o/err; exit 1; }
for w in 2 8; do
  timeout -k 10 200 python tools/bench_mo.py --algo moead --simulate-rank 0 --world $w > $o/moead_sim$w.json 2>>$o/err || { tail $o/err; exit 1; }
done
timeout -k 10 300 python tools/bench_neuro.py --pop 1024 --cap 1000 --graph > $o/ant_1024.json 2>>$o/err || { tail $o/err; exit 1; }
timeout -k 10 300 python tools/bench_neuro.py --pop 8192 --cap 1000 --graph > $o/ant_8192.json 2>>$o/err || { tail $o/err; exit 1; }
for f in nsga2 moead_1 moead_sim2 moead_sim8 ant_1024 ant_8192; do echo "$f $(tail -1 $o/$f.json | cut -c1-400)"; done
