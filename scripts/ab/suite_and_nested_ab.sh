set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 CONFIGS="nested" LIBS="head:fury_amd/lib_ab/libfory_rowfmt_head.so" bash scripts/ab_builds.sh
