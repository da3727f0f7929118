cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in libcauseweave_base.so libcauseweave.so; do
    CW_LIB=$PWD/cause_amd/$lib timeout -k 10 200 python bench.py --config 1 --steps 20 --warmup 5 > gpurun_out/c1_$lib.$rep.json 2> gpurun_out/c1_err.log || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['kernels_ms_per_step'].items()})" gpurun_out/c1_$lib.$rep.json
  done
done
