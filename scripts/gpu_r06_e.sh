# Round 6, call E: the Syn-1M step timeline after the host-loop fix; the sorted row-gradient plan (one rocPRIM
# radix sort, hvae_rgsort.hip) against the atomic plan at B = 4096 now that the host keeps ahead of the device
# (HVAE_RG_SORTED in the A/B library, alternating), Syn-1M and the Syn-10M shard.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_syn1m -o run -- \
  python3 $R/bench.py --workload syn1m --steps 150 --warmup 20 --no-cpu-baseline --probe-steps 2 > $O/kt_syn1m.log 2>&1 || exit 1
cd $R
python3 scripts/step_timeline.py $(find $O/kt_syn1m -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_syn1m.txt || exit 2
for r in 1 2; do
  for s in 0 1; do
    for wl in syn1m syn10m; do
      HVAE_LIB=build_var/libhvae_ab.so HVAE_RG_SORTED=$s timeout -k 10 300 python -u bench.py --workload $wl --steps 150 \
        --warmup 30 --no-cpu-baseline --probe-steps 2 2>> $O/bench.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'sorted':$s,'workload':'$wl','round':$r,'ms':d['ms_per_step'],'value':d['value']}))" >> $O/sorted_ab.jsonl || exit 3
    done
  done
done
echo done > $O/done
