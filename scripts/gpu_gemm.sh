# Per-shape timing of libhvae's fp32 GEMM at B = 4096 and B = 64 (scripts/bench_gemm.py).
set -e
mkdir -p gpurun_out
timeout -k 10 200 python scripts/bench_gemm.py --batch 4096 --reps 50 2>&1 | grep -v amdgpu.ids > gpurun_out/gemm4096.log
timeout -k 10 200 python scripts/bench_gemm.py --batch 64 --reps 100 2>&1 | grep -v amdgpu.ids > gpurun_out/gemm64.log
