# A/B of config 4 (maps) between two library builds on one box
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in libcauseweave_base.so libcauseweave.so; do
    CW_LIB=$PWD/cause_amd/$lib timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --check > gpurun_out/c4_$lib.$rep.json 2> gpurun_out/c4_err.log || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],4), d.get('kernel_sum_ms_per_step'), (d.get('check') or {}).get('mismatches'))" gpurun_out/c4_$lib.$rep.json
  done
done
