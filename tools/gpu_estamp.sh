set -o pipefail
for k in 21 63 77 99; do
  MHMKC_LIB=exp/libmhmkc_estamp.so timeout -k 10 200 python bench.py --k $k --steps 2 --warmup 1 --no-cpu-baseline --h2d-steps 0 --kmermap-sample-rows 0 > gpurun_out/estamp_k$k.log 2>&1 || { echo "k=$k failed"; tail -5 gpurun_out/estamp_k$k.log; exit 1; }
  echo "k=$k $(grep 'extract stamps' gpurun_out/estamp_k$k.log | tail -n 1)"
done
