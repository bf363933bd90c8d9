set -o pipefail
OUT=gpurun_out/r6af; mkdir -p $OUT
for x in 1 0 1 0; do
  timeout -k 10 300 python -u bench.py --workload c5 --steps 8 --warmup 3 --no-cpu --tune stream_priority=$x > $OUT/c5_prio$x.$RANDOM.json 2>> $OUT/c5.err || exit 1
done
JNI_HEAPS=auto JNI_SPECS="encode:6:3:1048576:4 encode:6:3:1048576:16 decode:6:3:1048576:4" JNI_TUNES="stream_priority=1 stream_priority=0 stream_priority=1 stream_priority=0 stream_priority=1 stream_priority=0" scripts/gpu_r6.sh r6af jnisweep
