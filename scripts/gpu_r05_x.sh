# decoder finalize in 16-B column form: decoder / train / large-step / API parity, then the Syn-1M and Syn-10M lines
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05x
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_api.py \
  tests/test_gpu_large_step.py tests/test_gpu_fp8.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 \
  || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for a in "--workload syn1m" "--precision bf16"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 300 python -u bench.py $a --steps 200 --warmup 20 --no-cpu-baseline \
    > $O/bench_$n.json 2> $O/bench_$n.err
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]);print(sys.argv[2],d['ms_per_step'],{k:v['us_per_step'] for k,v in d['launch_us'].items()})" $O/bench_$n.json $n
done
