cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/evry
for rep in 1 2; do for e in 4 1; do
timeout -k 10 240 python bench.py --steps 100 --warmup 10 --no-cpu --dropin-batches 0 --profile-every $e > gpurun_out/evry/e${e}_$rep.json 2>gpurun_out/evry/e${e}_$rep.err || exit 1
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('every',sys.argv[2], d['ms_per_step'], r['avg_launch_ms'], r['launches'], r['frac'])" gpurun_out/evry/e${e}_$rep.json $e
done; done
