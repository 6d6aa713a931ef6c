# Kernel trace of scripts/bench_gemm.py at the Syn-10M shapes (B = 4096, d = 768): hvae vs torch.mm kernel times
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/scripts/bench_gemm.py \
  --batch 4096 --d 768 --reps 50 > $O/bench_gemm.log 2>&1
tail -9 $O/bench_gemm.log
