#!/bin/bash
# Persistent vs one-group backward (tools/bwd_only.py, graph-replayed lv_group_action_bwd)
# across batches; A/B through the A/B library's LV_BWD_PERSIST_MIN (0 = off, 1 = always).
set -u
cd "$(dirname "$0")/.."
AB=lie-vae_amd/lie_vae/liblievae_hip_ab.so
for B in ${BATCHES:-4096 9216 16384 32768 65536 262144}; do
  for mode in default off on; do
    case $mode in
      default) ENVS="" ;;
      off) ENVS="LIEVAE_HIP_LIB=$AB LV_BWD_PERSIST_MIN=0" ;;
      on) ENVS="LIEVAE_HIP_LIB=$AB LV_BWD_PERSIST_MIN=1" ;;
    esac
    r=$(env $ENVS timeout -k 5 60 python tools/bwd_only.py $B 20 2>/dev/null | tail -1) || { echo "FAIL $B $mode"; exit 1; }
    echo "B=$B mode=$mode $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("us_per_call %.2f tile %d blocks %d" % (d["us_per_call"], d["plan"]["tile"], d["plan"]["blocks"]))')"
  done
done
