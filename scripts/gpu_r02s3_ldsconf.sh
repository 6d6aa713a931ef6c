# LDS bank-conflict census of every hot kernel: one PMC pass per workload (Syn-1M bf16 step: k_dec2_bf16, encoder,
# GEMMs, optimizer, row-gradient kernels; Syn-10M fp8 step: k_dec_fp8 d = 768 ring; fused top-K eval at Syn-1M).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ldsconf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/s1m -o run -- python3 $R/bench.py --workload syn1m --steps 5 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/s1m.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/f8 -o run -- python3 $R/bench.py --precision fp8 --steps 3 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/f8.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/tk -o run -- python3 $R/scripts/bench_eval.py --workload syn1m --probes topk_fused --skip-matrix --reps 2 > $O/tk.log 2>&1
python3 $R/scripts/pmc_summary.py $O/s1m > $O/s1m_summary.txt
python3 $R/scripts/pmc_summary.py $O/f8 > $O/f8_summary.txt
python3 $R/scripts/pmc_summary.py $O/tk > $O/tk_summary.txt
