# Round 6, call K: the deferred W1t update in the data-parallel W = 8 emulation (bf16, fp8; off vs the pending rows
# beside the finalize), and the Syn-10M lines once more (off / sweep, alternating).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06k
mkdir -p $O
cd $R
for P in fp8 bf16; do
  for arm in off sweep; do
    d=0; [ $arm = sweep ] && d=1
    HVAE_ADAM_DEFER=$d HVAE_DEFER_AT=sweep timeout -k 10 400 python3 -u scripts/bench_dp_emul.py --world 8 --steps 60 \
      --warmup 10 --precision $P > $O/emul_${P}_$arm.log 2>&1 || exit 1
  done
done
for r in 1 2; do
  for pr in fp8 bf16; do
    for arm in off sweep; do
      d=0; [ $arm = sweep ] && d=1
      HVAE_ADAM_DEFER=$d HVAE_DEFER_AT=sweep timeout -k 10 300 python -u bench.py --workload syn10m --precision $pr \
        --steps 150 --warmup 30 --no-cpu-baseline --probe-steps 2 2>> $O/bench.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'arm':'$arm','precision':'$pr','round':$r,'ms':d['ms_per_step']}))" >> $O/defer_ab.jsonl || exit 2
    done
  done
done
echo done > $O/done
