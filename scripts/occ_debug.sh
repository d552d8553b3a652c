KD_DEBUG_OCC=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline 2>&1 | grep -i "occupancy" | head -3
