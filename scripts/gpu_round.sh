mkdir -p gpurun_out
DEFAULT_SWEEP='[{}]'
SWEEP="${SWEEP:-$DEFAULT_SWEEP}"
timeout -k 10 600 python -m pytest tests -q -m gpu --ignore=tests/test_gpu_maps.py > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "lists rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_gpu_maps.py -q -x > gpurun_out/pytest_maps.log 2>&1; rc=$?
echo "maps rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python scripts/sweep.py "$SWEEP" --check > gpurun_out/sweep.log 2>&1; echo "sweep rc=$?"
