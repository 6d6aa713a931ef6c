# (1) the fp8 bench line at --probe-steps 5 after the probe's unarmed eager warm-up, (2) 99-negative eval throughput
# with the sampler's producer thread, (3) an SQ pass of the LDS-DMA GEMMs at the Syn-10M shapes
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05bb
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --precision fp8 --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline \
  > $O/bench_fp8.json 2> $O/bench_fp8.err
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]);print(d['ms_per_step'],{k:v['avg_us'] for k,v in d['launch_us'].items()})" $O/bench_fp8.json
timeout -k 10 400 python -u scripts/bench_eval.py --workload all_beauty > $O/eval_all_beauty.jsonl 2> $O/eval.err
grep neg99 $O/eval_all_beauty.jsonl
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_gemm' --output-format csv -d $O/gemm_sq -o run -- \
  python3 $R/scripts/bench_gemm.py --batch 4096 --d 768 --reps 5 --no-torch > $O/gemm_sq.log 2>&1
python3 $R/scripts/pmc_summary.py $O/gemm_sq > $O/gemm_sq_summary.txt
head -40 $O/gemm_sq_summary.txt
