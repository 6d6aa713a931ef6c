#!/bin/bash
# round 4 pass e: fp8 register-staging A/B (DEC5F8_RSTAGE 1 / 2) with its parity, the W = 8 rank-step emulation's
# kernel trace, and the product bench lines with the lazy-Adam sweep period 32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04e
mkdir -p $O
R=$GRAFT_REPO_ROOT
echo "fp8 rstage parity"
HVAE_LIB=$R/build_var/libhvae_f8rs2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_fp8.py tests/test_gpu_large.py -k "fp8" > $O/pytest_f8rs2.log 2>&1
rc=$?; tail -3 $O/pytest_f8rs2.log; [ $rc -eq 0 ] || exit $rc
echo "fp8 rstage A/B"
for round in 1 2; do
  for a in f8abl0 f8rs1 f8rs2; do
    HVAE_LIB=$R/build_var/libhvae_$a.so timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 \
      --dtype fp8 --reps 5 --ab DUMMY=$a --rounds 1 >> $O/f8_rs_ab.jsonl 2>> $O/f8_rs_ab.log || exit 3
  done
done
cut -c1-200 $O/f8_rs_ab.jsonl
echo "lazy adam tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  tests/test_gpu_large.py -k "lazy or train" > $O/pytest_lazy.log 2>&1
rc=$?; tail -3 $O/pytest_lazy.log; [ $rc -eq 0 ] || exit $rc
echo "emul trace"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/emul_kt -o run -- python3 $R/scripts/bench_dp_emul.py --world 8 --steps 10 --warmup 4 > $R/$O/emul_kt.log 2>&1 || exit 4
tail -2 $R/$O/emul_kt.log
cd $R
echo "benches"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline > $O/bench_syn10m.json 2> $O/bench_syn10m.log || exit 5
cut -c1-200 $O/bench_syn10m.json
timeout -k 10 300 python -u bench.py --workload syn1m --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log || exit 6
cut -c1-200 $O/bench_syn1m.json
timeout -k 10 300 python -u bench.py --workload all_beauty --steps 400 --warmup 40 --no-cpu-baseline > $O/bench_ab.json 2> $O/bench_ab.log || exit 7
cut -c1-200 $O/bench_ab.json
