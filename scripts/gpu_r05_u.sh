# LDS-DMA GEMM path with ring depth 2: GEMM / MLP / train-step parity, the Syn-10M shapes' kernel trace (product
# library beside torch.mm), then the bench lines of Syn-10M (bf16, fp8) and Syn-1M
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05u
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp_rows.py tests/test_gpu_train.py -x -q \
  --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/scripts/bench_gemm.py \
  --batch 4096 --d 768 --reps 50 > $O/bench_gemm.log 2>&1
python3 $R/scripts/gemm_trace_summary.py $O/tr/run_kernel_trace.csv | tee $O/gemm.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr384 -o run -- python3 $R/scripts/bench_gemm.py \
  --batch 4096 --d 384 --reps 50 > $O/bench_gemm384.log 2>&1
python3 $R/scripts/gemm_trace_summary.py $O/tr384/run_kernel_trace.csv | tee $O/gemm384.jsonl
HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_GEMM_DMA=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d $O/tr384_old -o run -- python3 $R/scripts/bench_gemm.py --batch 4096 --d 384 --reps 50 --no-torch \
  > $O/bench_gemm384_old.log 2>&1
python3 $R/scripts/gemm_trace_summary.py $O/tr384_old/run_kernel_trace.csv | tee $O/gemm384_old.jsonl
cd $R
for a in "--precision bf16" "--precision fp8" "--workload syn1m"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 300 python -u bench.py $a --steps 200 --warmup 20 --no-cpu-baseline \
    > $O/bench_$n.json 2> $O/bench_$n.err
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]);print(sys.argv[2],d['ms_per_step'],{k:v['us_per_step'] for k,v in d['launch_us'].items()})" $O/bench_$n.json $n
done
