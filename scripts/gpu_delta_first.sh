cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "delta" --timeout 120 --timeout-method thread -x > gpurun_out/gpu_delta.log 2>&1
rc=$?; echo "delta tests rc=$rc"; tail -15 gpurun_out/gpu_delta.log
if [ $rc -ne 0 ]; then exit $rc; fi
SKIP_BENCH=1 bash scripts/gpu_session.sh
