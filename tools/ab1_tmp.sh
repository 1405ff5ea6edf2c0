set -o pipefail
bash tools/ab_env.sh "base|X=1" "stamp|MHMKC_LIB=exp/libmhmkc_stamp.so MHMKC_PRINT_STAMPS=1" || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 -d $GRAFT_REPO_ROOT/gpurun_out/pcs -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --h2d-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/pcs.log 2>&1; echo "pcs rc=$?"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pcs.log; find $GRAFT_REPO_ROOT/gpurun_out/pcs -type f | head; du -sh $GRAFT_REPO_ROOT/gpurun_out/pcs
