#!/bin/bash
# GPU-box session 18: how HSA_CU_MASK bits map onto the MI355X's XCDs/CUs
# (census of the CUs a masked queue can use), before CU-partitioned replicas
# rely on it. Every mask tried keeps at least one CU on every XCD under both
# candidate mappings (bit i -> XCD i%8, or bit i -> XCD i/32), so no XCD is
# left without CUs.
set -o pipefail
out=gpurun_out/s18
mkdir -p $out
P=build/probe/amdgpu-dp-probe
run() {  # name mask
  if [ -z "$2" ]; then
    timeout -k 5 60 $P --device 0 --census > $out/census_$1.json 2> $out/census_$1.err
  else
    HSA_CU_MASK="$2" timeout -k 5 60 $P --device 0 --census > $out/census_$1.json 2> $out/census_$1.err
  fi
  rc=$?
  python3 -c "import json; d=json.load(open('$out/census_$1.json')); print('$1', repr('$2'), 'cus', d['cus'], 'seen', d['cus_seen'], 'xccs', d['xccs_seen'], 'per_xcc', d['per_xcc'])" || true
  return $rc
}
run full "" || exit 1
run all "0:0-255" || exit 1
# 8 bits in each 32-bit block plus 8..15: interleaved -> 9 CUs per XCD;
# blocked -> 16 on XCD 0 and 8 on the others.
run probe "0:0-15,32-39,64-71,96-103,128-135,160-167,192-199,224-231" || exit 1
python3 - <<'PY' > $out/mapping.txt
import json
d = json.load(open("gpurun_out/s18/census_probe.json"))
per = d["per_xcc"]
print("interleaved" if per and all(c == 9 for c in per) else ("blocked" if per and per[0] == 16 else "unknown:" + str(per)))
PY
m=$(cat $out/mapping.txt); echo mapping=$m
if [ "$m" = "interleaved" ]; then
  for r in 0 1 2 3; do run r4_$r "0:$((r*64))-$((r*64+63))" || exit 1; done
  for r in 0 7; do run r8_$r "0:$((r*32))-$((r*32+31))" || exit 1; done
  run r32_0 "0:0-7" || exit 1
  run r32_31 "0:248-255" || exit 1
  python3 - <<'PY'
import json
ks = [set(json.load(open(f"gpurun_out/s18/census_r4_{r}.json"))["keys"]) for r in range(4)]
full = set(json.load(open("gpurun_out/s18/census_full.json"))["keys"])
print("r4 disjoint:", all(not (ks[a] & ks[b]) for a in range(4) for b in range(a + 1, 4)),
      "union == full:", set().union(*ks) == full, [len(k) for k in ks])
PY
fi
