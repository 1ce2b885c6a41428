# 2-rank gloo rehearsal of bench.py in two trees (current, _bisect) to locate a DP slowdown
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for tree in _bisect .; do
( cd $tree && timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu > /tmp/dp2.json 2> /tmp/dp2.err ) || { tail -30 /tmp/dp2.err; exit 1; }
python3 -c "import json; l=[x for x in open('/tmp/dp2.json') if x.startswith('{')][0]; d=json.loads(l); print('$tree', d['value'], d['ms_per_step'], d['phases_ms_per_launch'].get('stft_mel'), d['phases_ms_per_launch'].get('conv2_fwd'))"
done
