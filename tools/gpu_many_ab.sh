set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_etf.py -m gpu -k "from_binary" -x -q --timeout 120 --timeout-method thread > gpurun_out/many_tests.log 2>&1
rc=$?; tail -5 gpurun_out/many_tests.log; [ $rc -eq 0 ] || exit $rc
KS=4,32,64 AB_CMD=tools/decoder_probe.py bash tools/gpu_ab_lib.sh
