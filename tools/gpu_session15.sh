#!/bin/bash
# GPU-box session 15: rocprofv3 PMC counters for the probe kernels, one counter
# per pass (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950), with
# --kernel-trace only (no sys/runtime traces).
set -o pipefail
out=gpurun_out/s15
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || { echo BUILD FAILED; tail -30 $out/build.log; exit 1; }
cd /tmp
P=$GRAFT_REPO_ROOT/build/probe/amdgpu-dp-probe
for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU_MFMA_BF16; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -f csv -d $GRAFT_REPO_ROOT/$out/pmc_$c -o probe -- $P --device 0 --bytes 1073741824 --iters 3 --mfma > $GRAFT_REPO_ROOT/$out/pmc_$c.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$out/pmc_$c.log; exit 1; }
  echo "== $c"; find $GRAFT_REPO_ROOT/$out/pmc_$c -name "*counter_collection*.csv" | head -2
done
