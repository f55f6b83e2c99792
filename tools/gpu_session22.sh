#!/bin/bash
# GPU-box session 22: noisy-neighbour interference on one MI355X, with and
# without CU shares (what --replica-cu-mask buys a latency-sensitive pod).
# Victim: 2000 launches of a small kernel, host-timed. Aggressor: a second
# process saturating the GPU with 1 ms kernels for 8 s.
set -o pipefail
out=gpurun_out/s22
mkdir -p $out
P=build/probe/amdgpu-dp-probe
lat() {  # name victim_mask aggressor_mask(or "none")
  if [ "$3" != "none" ]; then
    if [ -n "$3" ]; then HSA_CU_MASK="$3" timeout -k 5 40 $P --device 0 --aggressor 8 > $out/aggr_$1.json 2>&1 &
    else timeout -k 5 40 $P --device 0 --aggressor 8 > $out/aggr_$1.json 2>&1 & fi
    apid=$!
    sleep 1.5
  fi
  if [ -n "$2" ]; then HSA_CU_MASK="$2" timeout -k 5 60 $P --device 0 --latency 2000 > $out/lat_$1.json 2> $out/lat_$1.err
  else timeout -k 5 60 $P --device 0 --latency 2000 > $out/lat_$1.json 2> $out/lat_$1.err; fi
  rc=$?
  if [ "$3" != "none" ]; then wait $apid || { echo "aggressor failed"; cat $out/aggr_$1.json; return 1; }; fi
  echo "$1 victim_mask='$2' aggressor_mask='$3' $(cat $out/lat_$1.json)"
  return $rc
}
lat solo_full "" none || exit 1
lat solo_quarter "0:0-63" none || exit 1
lat shared_nomask "" "" || exit 1
lat shared_masked "0:0-63" "0:64-255" || exit 1
lat shared_victim_masked_only "0:0-63" "" || exit 1
