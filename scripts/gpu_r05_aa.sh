#!/bin/bash
# finalize: the O partials prefetched at kernel start (FIN_OPRE=1 variant) vs the product, in the Syn-1M and Syn-10M steps
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05aa
for r in 1 2; do
  for v in prod finopre; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    for w in syn1m syn10m; do
      HVAE_LIB=$lib timeout -k 10 300 python -u bench.py --workload $w --steps 100 --warmup 10 --probe-steps 20 \
        --no-cpu-baseline > gpurun_out/r05aa/b_${v}_${w}_$r.json 2>>gpurun_out/r05aa/err.log || exit 1
      python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]);print(sys.argv[2],d['ms_per_step'],d['launch_us']['decoder_finalize']['avg_us'])" gpurun_out/r05aa/b_${v}_${w}_$r.json "$v $w"
    done
  done
done
