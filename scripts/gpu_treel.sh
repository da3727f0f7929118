# A/B of the tree variants on one box (k_tree vs k_tree_l tiles and modes, front
# effective parents; TL_VARIANTS overrides the list),
# then smoke and the GPU tests.  Usage (on the box): bash scripts/gpu_treel.sh
set -e
mkdir -p gpurun_out
V='[{"CW_TREE_L":"0"},{"CW_TREE_L":"2048"},{"CW_TREE_L":"1024"},{"CW_TL_MODE":"1"},{"CW_FRONT_EFF":"1"}]'
timeout -k 10 400 python -u scripts/sweep.py "${TL_VARIANTS:-$V}" --check --rounds 3 > gpurun_out/ab_treel.log 2>&1
echo ab-ok
CW_TREE_PROF=1 timeout -k 10 200 python -u scripts/sweep.py '[{"CW_TREE_L":"2048"}]' --rounds 1 > gpurun_out/prof_treel.log 2>&1
echo prof-ok
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
echo smoke-ok
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo tests-ok
