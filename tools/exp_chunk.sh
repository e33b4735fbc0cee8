# wavefront chunk-size sweep (paths per chunk)
for c in 4194304 8388608 16777216; do
  echo "chunk=$c $(MH_WF_CHUNK=$c timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"fwd_kernel_ms": [0-9.]*\|"bwd_kernel_ms": [0-9.]*' | tr '\n' ' ')"
done
