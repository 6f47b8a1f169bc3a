set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/gpu_tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc2=$?; echo "smoke rc=$rc2"; tail -5 gpurun_out/smoke.log
  if [ $rc2 -le 1 ]; then
    timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
    echo "bench rc=$?"; tail -5 gpurun_out/bench.log
  fi
fi
