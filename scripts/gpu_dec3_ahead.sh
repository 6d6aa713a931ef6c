# v3 operand read-ahead depth A/B (GEMM1 k-groups, GEMM2 d-blocks) at the Syn-10M shard shape.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ahead
mkdir -p $O
DEC="scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10"
for r in 1 2; do
for v in base g1a3 g1a4 g2a1 g2a3 g2a4 g13g23; do
  if [ $v = base ]; then L=""; else L="HVAE_LIB=$R/build_var/libhvae_$v.so"; fi
  env $L timeout -k 10 120 python $DEC > $O/$v.json 2>$O/$v.err && sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" $O/$v.json >> $O/all.jsonl
done
done
