# Round 6: the headline step (ultrasonic, f32split) at per-GPU batches 256 / 512 / 1024 / 2048 on one
# GPU -- throughput against batch (the bench line and the metric stay at configs[1]'s 512).
mkdir -p gpurun_out/r6_batch
for b in ${BATCHES:-256 512 1024 2048}; do
  timeout -k 10 300 python bench.py --batch $b --n-train $((16 * b)) --steps 100 --warmup 20 --no-cpu --dropin-batches 0 \
    > gpurun_out/r6_batch/b$b.json 2> gpurun_out/r6_batch/b$b.err || exit 1
  python -c "import json; d = json.load(open('gpurun_out/r6_batch/b$b.json')); print($b, d['ms_per_step'], round(d['value']), d['phases_ms_per_launch']['stft_mel'], d['phases_ms_per_launch']['conv2_fwd'])"
done
