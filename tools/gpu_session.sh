#!/bin/bash
# One parameterised GPU-box session (replaces round 1's gpu_check*.sh and
# gpu_session<N>.sh one-offs). Usage, from the repo root on the box:
#
#   OUT=gpurun_out/<name> bash tools/gpu_session.sh <step> [<step> ...]
#
# Steps (run in the order given; the session stops at the first failure, and
# every GPU step runs under its own `timeout -k`):
#   build        compile every native artefact (only needed if the tree was
#                shipped without build/; normally built on the CPU side)
#   tests        pytest -m gpu (thread-method timeouts, so a hang names its test)
#   smoke        __graft_entry__.smoke()
#   events       real amdsmi events (KFD PROCESS_START/END from the HIP probe):
#                raw, in-process and through the relay (tests/test_gpu_events.py);
#                records in gpurun_out/r6/
#   bench        the driver-shaped headline run (python bench.py, defaults)
#   configs      bench for the three real-hardware configs (spx-none,
#                timeslice4, auto-mem), 50 steps each
#   health       the GPU tests for health liveness (events on/off and why, first
#                ECC poll) and the partition APIs; evidence in gpurun_out/health/
#   partition    what libamd_smi reports for the partition APIs (JSON)
#   prof         rocprofv3 --kernel-trace --stats of the HIP probe (copy, MFMA,
#                census, latency kernels)
#   pmc          rocprofv3 --pmc, one counter per pass (FETCH_SIZE, WRITE_SIZE,
#                SQ_INSTS_VALU_MFMA_BF16)
#   census       HSA_CU_MASK -> XCD/CU census of the probe (quarter shares)
#   interference noisy-neighbour victim latency with and without CU shares
#   unitslots    the interference pair for two packed 36 GB memory-unit pods,
#                proportional (one shared CU slot) vs --memory-unit-cu-slots whole
#   floor        UDS ping-pong floor, busy-poll on and off
#   spread       10 back-to-back headline runs (bench.py --no-probe); line:
#                R i p50 p99 grpc-go grpcio pods/s relation client_cpu loop_cpu
#                residency_p50 residency_p99 (the daemon's read -> reply time)
#   access       device-cgroup denial (EPERM on /dev/kfd, /dev/dri/*, the
#                errno an unprivileged pod's device cgroup returns) through
#                libadp_devcgroup_sim.so: --smi-report / --dry-run / the
#                health monitor's log, with and without the denial
#   driver       what the driver reports per process (KFD sysfs, DRM fdinfo,
#                amdsmi_get_gpu_process_list) while PyTorch holds HBM
#   ab           interleaved headline runs per --loop-affinity mode (AB_MODES,
#                default "none peer-l3"; AB_PAIRS rounds, default 8), plus the
#                8-rank mock node (AB_RANKS) per mode
#   cpus         the CPUs this box lets the session use, grouped by L3 / NUMA
#   curve        tools/mock_curve.sh (CONFIGS="spx-none" for one config)
#   idle         the daemon's idle footprint on real libamd_smi (CPU, wake-ups,
#                RSS; default config and memory units enforced), IDLE_SECONDS (60)
#   soak         SOAK_SECONDS (default 180) of churn + SIGHUP + kubelet restarts + scrapes on
#                real libamd_smi (health polling, state file): RSS/fd/thread leaks
set -o pipefail
out=${OUT:-gpurun_out/session}
mkdir -p "$out"
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
P=$ROOT/build/probe/amdgpu-dp-probe

die() { echo "$1 FAILED"; [ -n "$2" ] && tail -40 "$2"; exit 1; }

step_build() {
  timeout -k 10 600 python -c "import __graft_entry__ as g; g.build()" > $out/build.log 2>&1 || die build $out/build.log
  echo built
}
step_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || die "GPU TESTS" $out/pytest_gpu.log
  tail -2 $out/pytest_gpu.log
}
step_events() {
  timeout -k 10 600 python -u -m pytest tests/test_gpu_events.py -m gpu -v -rs --timeout 180 --timeout-method thread \
    -p no:cacheprovider > $out/pytest_events.log 2>&1 || die EVENTS $out/pytest_events.log
  tail -4 $out/pytest_events.log
}
step_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.json 2> $out/smoke.err || die SMOKE $out/smoke.err
  tail -1 $out/smoke.json
}
step_bench() {
  timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err || die BENCH $out/bench_default.err
  cat $out/bench_default.json
}
step_configs() {
  for cfg in spx-none timeslice4 auto-mem auto-mem-enforced; do
    timeout -k 10 300 python bench.py --steps 50 --warmup 5 --config $cfg > $out/bench_$cfg.json 2> $out/bench_$cfg.err || die "BENCH $cfg" $out/bench_$cfg.err
    python -c "import json; d=json.load(open('$out/bench_$cfg.json')); print('$cfg', d['allocatable'], d['value'], d['allocate_p99_us'], d['preferred_p50_us'], d['server_allocate_handler_avg_us'], d.get('grpc_go_shaped_allocate_p50_us'), d.get('grpcio_client_allocate_p50_us'), d['pods_per_s'])"
  done
}
step_health() {
  # The GPU tests that check health liveness and record the partition APIs keep
  # their evidence in gpurun_out/health/ (daemon log, partition_apis.json).
  timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "health or partition_profile" > $out/health.log 2>&1 || die HEALTH $out/health.log
  grep -h "health poll #1\|event notification" gpurun_out/health/daemon_real_amdsmi_health.log || true
}
step_partition() {
  timeout -k 10 60 python -c "import json; from k8s_gpu_sharing_plugin_amd.utils import native; print(json.dumps(native.snapshot(), indent=1))" > $out/snapshot.json 2> $out/snapshot.err || die PARTITION $out/snapshot.err
  python -c "import json; d=json.load(open('$out/snapshot.json')); g=d['gpus'][0]; print({k: g.get(k) for k in ('bdf','vram_mib','vram_source','driver_profile','compute_mode','memory_mode','profile','model_hbm_mib')}); print([p.get('reported') for p in g['partitions']][:8])"
}
step_prof() {
  ( cd /tmp && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $ROOT/$out/prof -o probe -- $P --device 0 --bytes 1073741824 --iters 3 --mfma > $ROOT/$out/prof.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $ROOT/$out/prof_census -o census -- $P --device 0 --census > $ROOT/$out/prof_census.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $ROOT/$out/prof_latency -o latency -- $P --device 0 --latency 500 > $ROOT/$out/prof_latency.log 2>&1 ) || die PROF $out/prof.log
  find $out -name "*kernel_stats.csv" -exec cat {} \;
}
step_pmc() {
  for c in FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU_MFMA_BF16; do
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -f csv -d $ROOT/$out/pmc_$c -o probe -- $P --device 0 --bytes 1073741824 --iters 3 --mfma > $ROOT/$out/pmc_$c.log 2>&1 ) || die "PMC $c" $out/pmc_$c.log
    echo "== $c"; find $out/pmc_$c -name "*counter_collection*.csv" | head -2
  done
}
census_one() {  # name mask
  if [ -z "$2" ]; then timeout -k 5 60 $P --device 0 --census > $out/census_$1.json 2> $out/census_$1.err
  else HSA_CU_MASK="$2" timeout -k 5 60 $P --device 0 --census > $out/census_$1.json 2> $out/census_$1.err; fi || die "CENSUS $1" $out/census_$1.err
  python3 -c "import json; d=json.load(open('$out/census_$1.json')); print('$1', repr('$2'), 'cus', d['cus'], 'seen', d['cus_seen'], 'xccs', d['xccs_seen'], 'per_xcc', d['per_xcc'])"
}
step_census() {
  census_one full ""
  for r in 0 1 2 3; do census_one r4_$r "0:$((r*64))-$((r*64+63))"; done
}
lat_one() {  # name victim_mask aggressor_mask(or "none")
  local apid=
  if [ "$3" != "none" ]; then
    if [ -n "$3" ]; then HSA_CU_MASK="$3" timeout -k 5 40 $P --device 0 --aggressor 8 > $out/aggr_$1.json 2>&1 &
    else timeout -k 5 40 $P --device 0 --aggressor 8 > $out/aggr_$1.json 2>&1 & fi
    apid=$!
    sleep 1.5
  fi
  if [ -n "$2" ]; then HSA_CU_MASK="$2" timeout -k 5 60 $P --device 0 --latency 2000 > $out/lat_$1.json 2> $out/lat_$1.err
  else timeout -k 5 60 $P --device 0 --latency 2000 > $out/lat_$1.json 2> $out/lat_$1.err; fi || die "LATENCY $1" $out/lat_$1.err
  if [ -n "$apid" ]; then wait $apid || die "AGGRESSOR $1" $out/aggr_$1.json; fi
  echo "$1 victim_mask='$2' aggressor_mask='$3' $(cat $out/lat_$1.json)"
}
step_interference() {
  lat_one solo_full "" none
  lat_one solo_quarter "0:0-63" none
  lat_one shared_nomask "" ""
  lat_one shared_masked "0:0-63" "0:64-255"
}
step_unitslots() {
  # Two packed 36 GB memory-unit pods (the masks tests/test_e2e_mock.py pins):
  # proportional shares slot 3 (CUs 24-31), --memory-unit-cu-slots whole not.
  lat_one units_prop_solo "0:0-31" none
  lat_one units_prop_shared "0:0-31" "0:24-63"
  lat_one units_whole_solo "0:0-23" none
  lat_one units_whole_shared "0:0-23" "0:32-55"
}
step_floor() {
  for b in 50 0; do
    timeout -k 10 120 build/native/amdgpu-dp-uds-floor --iters 200000 --busy-poll-us $b > $out/floor_bp$b.json || die FLOOR
    cat $out/floor_bp$b.json
  done
}
step_spread() {
  for i in $(seq 1 10); do
    timeout -k 10 300 python bench.py --no-probe > $out/spread_$i.json 2> $out/spread_$i.err || die "SPREAD $i" $out/spread_$i.err
    python -c "import json; d=json.load(open('$out/spread_$i.json')); p=d.get('placement') or {}; print('R $i', d['value'], d['allocate_p99_us'], d.get('grpc_go_shaped_allocate_p50_us'), d.get('grpcio_client_allocate_p50_us'), d['pods_per_s'], p.get('relation'), p.get('client_cpu'), p.get('busiest_loop_cpu'), *[(r or {}).get(k) for r in [(d.get('server_residency') or {}).get('native_client')] for k in ('p50_us', 'p99_us')])"
  done
}
step_access() {
  local D=build/native/amdgpu-device-plugin SIM=$ROOT/build/native/libadp_devcgroup_sim.so
  local dp=$(mktemp -d /tmp/adpacc-XXXX)
  timeout -k 10 60 $D --device-plugin-path $dp --smi-report > $out/smi_report.json 2> $out/smi_report.err || die "SMI REPORT" $out/smi_report.err
  LD_PRELOAD=$SIM timeout -k 10 60 $D --device-plugin-path $dp --smi-report > $out/smi_report_denied.json 2> $out/smi_report_denied.err || die "SMI REPORT (denied)" $out/smi_report_denied.err
  ADP_DEVCGROUP_ALLOW=/dev/dri LD_PRELOAD=$SIM timeout -k 10 60 $D --device-plugin-path $dp --smi-report > $out/smi_report_kfd_denied.json 2> $out/smi_report_kfd_denied.err || die "SMI REPORT (kfd denied)" $out/smi_report_kfd_denied.err
  ADP_DEVCGROUP_ALLOW=/dev/kfd LD_PRELOAD=$SIM timeout -k 10 60 $D --device-plugin-path $dp --smi-report > $out/smi_report_dri_denied.json 2> $out/smi_report_dri_denied.err || die "SMI REPORT (dri denied)" $out/smi_report_dri_denied.err
  LD_PRELOAD=$SIM timeout -k 10 60 $D --device-plugin-path $dp --dry-run > $out/dry_run_denied.json 2> $out/dry_run_denied.err || die "DRY RUN (denied)" $out/dry_run_denied.err
  timeout -k 10 120 python tools/access_daemon_check.py $out/daemon_denied.log > $out/daemon_denied.txt 2>&1 || die "DAEMON (denied)" $out/daemon_denied.txt
  cat $out/daemon_denied.txt
  python3 tools/compare_smi_reports.py $out/smi_report.json $out/smi_report_denied.json $out/smi_report_kfd_denied.json $out/smi_report_dri_denied.json | tee $out/access_summary.txt
  rm -rf $dp
}
step_idle() {
  local secs=${IDLE_SECONDS:-60}
  timeout -k 10 $((secs + 90)) python tools/idle_footprint.py --real --seconds $secs > $out/idle.json 2> $out/idle.err || die IDLE $out/idle.err
  timeout -k 10 $((secs + 90)) python tools/idle_footprint.py --real --enforce --seconds $secs > $out/idle_enforce.json 2> $out/idle_enforce.err || die "IDLE (enforce)" $out/idle_enforce.err
  # the chart's layout: events and scans through the event relay
  timeout -k 10 $((secs + 90)) python tools/idle_footprint.py --real --enforce --relay --seconds $secs > $out/idle_relay.json 2> $out/idle_relay.err || die "IDLE (relay)" $out/idle_relay.err
  cat $out/idle.json $out/idle_enforce.json $out/idle_relay.json
}
step_driver() {
  timeout -k 10 180 python tools/probe_driver_usage.py > $out/driver_usage.json 2> $out/driver_usage.err || die DRIVER $out/driver_usage.err
  python3 -c "import json; d=json.load(open('$out/driver_usage.json')); print(json.dumps({'self_fdinfo': d.get('self_fdinfo'), 'child': {k: v for k, v in d['child'].items() if k != 'cgroup'}})[:3000])"
}
step_ab() {
  local modes=${AB_MODES:-none peer-l3} pairs=${AB_PAIRS:-8} port=29711
  for i in $(seq 1 $pairs); do
    for m in $modes; do
      DP_LOOP_AFFINITY=$m timeout -k 10 300 python bench.py --no-probe > $out/ab_${m}_$i.json 2> $out/ab_${m}_$i.err || die "AB $m $i" $out/ab_${m}_$i.err
      python -c "import json; d=json.load(open('$out/ab_${m}_$i.json')); print('AB $m $i', d['value'], d['allocate_p99_us'], d.get('grpc_go_shaped_allocate_p50_us'), d['pods_per_s'])"
    done
  done
  for i in $(seq 1 ${AB_RANK_PAIRS:-3}); do
    for m in $modes; do
      port=$((port + 1))
      DP_LOOP_AFFINITY=$m timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${AB_RANKS:-8} \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus ${AB_RANKS:-8} --mock --no-probe \
        > $out/abr_${m}_$i.json 2> $out/abr_${m}_$i.err || die "AB ranks $m $i" $out/abr_${m}_$i.err
      python -c "import json; d=json.loads(open('$out/abr_${m}_$i.json').read().strip().splitlines()[-1]); print('ABR $m $i', d['value'], d['allocate_p99_us'], d.get('grpc_go_shaped_allocate_p50_us'), d['pods_per_s'])"
    done
  done
}
step_cpus() {
  python3 tools/cpu_layout.py > $out/cpus.json || die CPUS
  cat $out/cpus.json
}
step_curve() {
  bash tools/mock_curve.sh $out/curve || die CURVE
}
step_soak() {
  local secs=${SOAK_SECONDS:-180}
  # one gpurun call may run 1200 s in all: leave room for the box set-up and the summary
  if [ "$secs" -gt 1000 ]; then echo "SOAK_SECONDS=$secs does not fit one call; using 1000"; secs=1000; fi
  timeout -k 10 $((secs + 220)) python -u tools/soak.py --seconds $secs --real ${SOAK_ARGS:-} --out $out/soak.json > $out/soak.log 2>&1 || die SOAK $out/soak.log
  tail -1 $out/soak.log
}

[ $# -gt 0 ] || set -- tests smoke bench prof
for s in "$@"; do
  declare -F step_$s > /dev/null || { echo "unknown step $s"; exit 2; }
  echo "== $s"
  step_$s
done
echo "session done"
