bash tools/gpu_r04_b.sh r04b
