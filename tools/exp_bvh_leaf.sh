# BVH leaf-size / SAH traversal-cost sweep for the packet engine (fwd step)
for L in 6 8 12 16 31; do for C in 4 100; do
  echo "leaf=$L ct=$C $(MH_BVH_LEAF=$L MH_BVH_CT=$C timeout -k 10 120 python bench.py --no-cpu --fwd-only --steps 3 --warmup 1 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_us": [0-9.]*' | tr '\n' ' ')"
done; done
echo "lane engine leaf=4: $(MH_TRAVERSAL=lane timeout -k 10 120 python bench.py --no-cpu --fwd-only --steps 3 --warmup 1 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' )"
echo "lane engine leaf=8 ct=4: $(MH_TRAVERSAL=lane MH_BVH_LEAF=8 MH_BVH_CT=4 timeout -k 10 120 python bench.py --no-cpu --fwd-only --steps 3 --warmup 1 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' )"
