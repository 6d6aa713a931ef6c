#!/bin/bash
# round 4 pass d: fp8 d = 768 sweep anatomy (DEC5F8_ABL arms), the lazy-Adam sweep period with the hardware-sqrt
# Adam (8 / 16 / 32), the Syn-10M GEMM shapes (libhvae vs torch.mm) and an SQ counter pass of the GEMM kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04d
mkdir -p $O
R=$GRAFT_REPO_ROOT
echo "fp8 anatomy"
for round in 1 2; do
  for a in 0 1 3 7 31 96 124 128 252; do
    HVAE_LIB=$R/build_var/libhvae_f8abl$a.so timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 \
      --dtype fp8 --reps 5 --ab DUMMY=f8abl$a --rounds 1 >> $O/f8_abl.jsonl 2>> $O/f8_abl.log || exit 3
  done
done
cat $O/f8_abl.jsonl | cut -c1-200
echo "sweep period"
for round in 1 2; do
  for a in base sweep16 sweep32; do
    lib=$R/build_var/libhvae_$a.so; [ $a = base ] && lib=$R/recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline > $O/bench_$a.json 2>> $O/bench_sweep.log || exit 4
    python3 -c "
import json; d=json.load(open('$O/bench_$a.json')); L=d['launch_us']
print(json.dumps({'arm': '$a', 'round': $round, 'ms_per_step': d['ms_per_step'], 'sweep_us': L['decoder_sweep']['avg_us'], 'adam_rows_us': L['adam_rows']['avg_us'], 'adam_catchup_us': L['adam_catchup']['avg_us']}))" >> $O/sweep_period.jsonl
  done
done
cat $O/sweep_period.jsonl
echo "gemm shapes"
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 768 --reps 50 > $O/gemm_syn10m.jsonl 2> $O/gemm_syn10m.log || exit 5
cat $O/gemm_syn10m.jsonl | cut -c1-250
echo "gemm sq"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_gemm' --output-format csv -d $R/$O/gemm_sq -o run -- python3 $R/scripts/bench_gemm.py --batch 4096 --d 768 --reps 4 --no-torch > $R/$O/gemm_sq.log 2>&1 || exit 6
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_gemm' --output-format csv -d $R/$O/gemm_kt -o run -- python3 $R/scripts/bench_gemm.py --batch 4096 --d 768 --reps 20 --no-torch > $R/$O/gemm_kt.log 2>&1 || exit 7
python3 $R/scripts/pmc_summary.py $R/$O/gemm_sq > $R/$O/gemm_sq_summary.txt 2>&1
head -60 $R/$O/gemm_sq_summary.txt
