# Developer entry points (the reference's Makefile: fmt/vet/lint/build/test/coverage).
BUILD      ?= build/native
JOBS       ?= 8
PY         ?= python3
GPURUN     ?= /usr/local/graft/bin/gpurun

.PHONY: all build probe test test-native test-gpu bench asan tsan tsan-e2e asan-e2e fuzz coverage analyze lint image image-rootfs clean

# Containerised targets (reference Makefile:44-74): `make docker-<target>` runs
# `make <target>` in the development image built from docker/Dockerfile.devel.
DOCKER        ?= docker
ROCM_VERSION  ?= 7.2
BUILDIMAGE    ?= amdgpu-device-plugin-build:rocm$(ROCM_VERSION)
DOCKER_TARGETS := $(patsubst %,docker-%,build test test-native lint asan tsan asan-e2e tsan-e2e coverage)
.PHONY: .build-image $(DOCKER_TARGETS)
.build-image: docker/Dockerfile.devel
	if [ -z "$(SKIP_IMAGE_BUILD)" ]; then \
	  $(DOCKER) build --build-arg ROCM_VERSION=$(ROCM_VERSION) --tag $(BUILDIMAGE) -f $< docker; \
	fi
$(DOCKER_TARGETS): docker-%: .build-image
	@echo "Running 'make $(*)' in docker container $(BUILDIMAGE)"
	$(DOCKER) run --rm -v $(CURDIR):$(CURDIR) -w $(CURDIR) --user $$(id -u):$$(id -g) \
	  -e HOME=/tmp $(BUILDIMAGE) make $(*)

all: build

build:
	cmake -S native -B $(BUILD) -G Ninja -DCMAKE_BUILD_TYPE=Release >/dev/null
	ninja -C $(BUILD) -j$(JOBS)

probe:
	$(PY) -c "from k8s_gpu_sharing_plugin_amd.utils import build; build.build_probe()"

# Unit tests, then the bounded model check of the health state machine: every
# sequence of up to HEALTH_MODEL_DEPTH steps over its 16 events, both layouts,
# then up to HEALTH_MODEL_EXT_DEPTH steps over the extended 24/25 events.
HEALTH_MODEL_DEPTH ?= 6
HEALTH_MODEL_EXT_DEPTH ?= 5
test-native: build
	$(BUILD)/adp_unit_tests
	$(BUILD)/adp_health_model --depth $(HEALTH_MODEL_DEPTH)
	$(BUILD)/adp_health_model --extended --depth $(HEALTH_MODEL_EXT_DEPTH)

test: build
	$(PY) -m pytest tests -q -m "not gpu"

# Real MI355X (one GPU box): GPU tests, smoke, bench, rocprof of the probe.
test-gpu:
	$(GPURUN) --timeout 1200 -- 'OUT=gpurun_out/check bash tools/gpu_session.sh tests smoke bench prof'

bench: build
	$(PY) bench.py --steps 20 --warmup 2

# Sanitizer builds of the native unit + stress tests (host code only).
asan:
	cmake -S native -B build/asan -G Ninja -DCMAKE_BUILD_TYPE=Debug -DADP_SANITIZE=ON >/dev/null
	ninja -C build/asan -j$(JOBS) adp_unit_tests adp_stress adp_health_model amdsmi_mock adp_memcap adp_memcap_check
	ASAN_OPTIONS=detect_leaks=1 build/asan/adp_unit_tests
	build/asan/adp_stress
	ASAN_OPTIONS=detect_leaks=1 build/asan/adp_health_model --depth 4
	ASAN_OPTIONS=detect_leaks=1 build/asan/adp_health_model --extended --depth 3
	LD_PRELOAD="$$(gcc -print-file-name=libasan.so) $(CURDIR)/build/asan/libadp_memcap.so" ASAN_OPTIONS=detect_leaks=0 \
	  AMD_GPU_MEMORY_LIMIT_MIB=100,50 ADP_MEMCAP_KEY=make-asan-$$$$ build/asan/adp_memcap_check
	LD_PRELOAD="$$(gcc -print-file-name=libasan.so) $(CURDIR)/build/asan/libadp_memcap.so" ASAN_OPTIONS=detect_leaks=0 \
	  AMD_GPU_MEMORY_LIMIT_MIB=40 ADP_MEMCAP_KEY=make-asan-stress-$$$$ build/asan/adp_memcap_check stress
	rm -f /dev/shm/adp-memcap-key-make-asan-*

tsan:
	cmake -S native -B build/tsan -G Ninja -DCMAKE_BUILD_TYPE=Debug -DADP_TSAN=ON >/dev/null
	ninja -C build/tsan -j$(JOBS) adp_unit_tests adp_stress amdsmi_mock adp_memcap adp_memcap_check
	TSAN_OPTIONS=halt_on_error=1 build/tsan/adp_unit_tests
	TSAN_OPTIONS=halt_on_error=1 build/tsan/adp_stress
	# the HBM-cap shim: 8 threads of allocations against a cap
	TSAN_OPTIONS=halt_on_error=1 LD_PRELOAD="$$(gcc -print-file-name=libtsan.so) $(CURDIR)/build/tsan/libadp_memcap.so" \
	  AMD_GPU_MEMORY_LIMIT_MIB=40 ADP_MEMCAP_KEY=make-tsan-$$$$ build/tsan/adp_memcap_check stress
	# stream-ordered allocations racing refusal-triggered pool trims
	TSAN_OPTIONS=halt_on_error=1 LD_PRELOAD="$$(gcc -print-file-name=libtsan.so) $(CURDIR)/build/tsan/libadp_memcap.so" \
	  AMD_GPU_MEMORY_LIMIT_MIB=100 ADP_MEMCAP_KEY=make-tsan-race-$$$$ build/tsan/adp_memcap_check poolrace
	TSAN_OPTIONS=halt_on_error=1 LD_PRELOAD="$$(gcc -print-file-name=libtsan.so) $(CURDIR)/build/tsan/libadp_memcap.so" \
	  AMD_GPU_MEMORY_LIMIT_MIB=100 ADP_MEMCAP_KEY=make-tsan-fork-$$$$ build/tsan/adp_memcap_check fork 60
	rm -f /dev/shm/adp-memcap-key-make-tsan-*

# The daemon itself under TSan, driven by the end-to-end suites (tests that load
# the C API into Python are skipped: a TSan .so cannot be dlopen'ed there).
tsan-e2e:
	cmake -S native -B build/tsan -G Ninja -DCMAKE_BUILD_TYPE=RelWithDebInfo -DADP_TSAN=ON >/dev/null
	ninja -C build/tsan -j$(JOBS) amdgpu-device-plugin amdgpu-dp-kubelet amdsmi_mock amdgpu-dp-event-probe
	rm -rf build/tsan-logs && mkdir -p build/tsan-logs
	ADP_BUILD_DIR=$(CURDIR)/build/tsan TSAN_OPTIONS=log_path=$(CURDIR)/build/tsan-logs/daemon \
	  $(PY) -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_e2e_mock.py tests/test_health.py \
	  tests/test_metrics.py tests/test_lifecycle.py tests/test_robustness.py tests/test_h2_native.py \
	  tests/test_health_persistence.py tests/test_h2_grpcgo.py tests/test_config.py tests/test_partition_shapes.py tests/test_driver_hbm.py tests/test_preferred.py \
	  tests/test_event_relay.py tests/test_policy_units.py tests/test_hip_order.py tests/test_kfd_topology.py tests/test_chart_layout.py \
	  tests/test_memory_unit_guards.py tests/test_parity_contract.py tests/test_metrics_exposition.py tests/test_gpu_recovery.py \
	  tests/test_event_matching.py tests/test_relay_protocol.py tests/test_lifecycle_chaos.py tests/test_relay_client.py \
	  -k "not additional_ids and not classification and not bruteforce and not snapshot_reports and not scan_reads_only and not another_namespace and not without_client_id and not partitions_read and not parser_edge and not hosted and not event_types_parse"
	@if ls build/tsan-logs/* >/dev/null 2>&1; then cat build/tsan-logs/*; exit 1; fi

# The daemon under ASan/UBSan/LSan, driven by the same end-to-end suites.
# Coverage-guided fuzzing (libFuzzer, ASan+UBSan, clang from ROCm's LLVM) of
# every parser that sees bytes from outside: the RPC handlers, HTTP/2, the
# protobuf codec, the config front end, grant accounting files + /metrics, the
# driver-side /proc scan (native/fuzz/). FUZZ_SECONDS per target, in parallel;
# corpora grow in build/fuzz/corpus/<target>; a crash leaves build/fuzz/crash-*.
FUZZ_TARGETS ?= plugin h2 h2_diff h2_client proto config grantfile procscan relay
FUZZ_SECONDS ?= 60
CLANGXX      ?= /opt/rocm/lib/llvm/bin/clang++
fuzz:
	cmake -S native -B build/fuzz -G Ninja -DCMAKE_BUILD_TYPE=RelWithDebInfo -DADP_FUZZ=ON \
	  -DCMAKE_CXX_COMPILER=$(CLANGXX) -DCMAKE_C_COMPILER=$(dir $(CLANGXX))clang >/dev/null
	ninja -C build/fuzz -j$(JOBS) $(addprefix fuzz_,$(FUZZ_TARGETS))
	$(PY) tools/gen_fuzz_seeds.py build/fuzz/corpus/h2 build/fuzz/corpus/h2_diff build/fuzz/corpus/h2_client
	cd build/fuzz && rm -f fuzz_*.failed && for t in $(FUZZ_TARGETS); do mkdir -p corpus/$$t; \
	  ( ./fuzz_$$t -max_total_time=$(FUZZ_SECONDS) -rss_limit_mb=2048 -print_final_stats=1 corpus/$$t \
	    > fuzz_$$t.log 2>&1 || echo "fuzz_$$t FAILED (build/fuzz/fuzz_$$t.log)" > fuzz_$$t.failed ) & done; wait; \
	  for t in $(FUZZ_TARGETS); do grep -h "DONE" fuzz_$$t.log | sed "s/^/$$t /"; done; \
	  ! cat fuzz_*.failed 2>/dev/null

asan-e2e:
	cmake -S native -B build/asan -G Ninja -DCMAKE_BUILD_TYPE=Debug -DADP_SANITIZE=ON >/dev/null
	ninja -C build/asan -j$(JOBS) amdgpu-device-plugin amdgpu-dp-kubelet amdsmi_mock amdgpu-dp-event-probe
	rm -rf build/asan-logs && mkdir -p build/asan-logs
	ADP_BUILD_DIR=$(CURDIR)/build/asan ASAN_OPTIONS=log_path=$(CURDIR)/build/asan-logs/daemon:detect_leaks=1:verify_asan_link_order=0 \
	  UBSAN_OPTIONS=print_stacktrace=1:log_path=$(CURDIR)/build/asan-logs/ubsan \
	  $(PY) -m pytest -q -p no:cacheprovider -m "not gpu" tests/test_e2e_mock.py tests/test_health.py \
	  tests/test_metrics.py tests/test_lifecycle.py tests/test_robustness.py tests/test_h2_native.py \
	  tests/test_health_persistence.py tests/test_h2_grpcgo.py tests/test_config.py tests/test_partition_shapes.py tests/test_driver_hbm.py tests/test_preferred.py \
	  tests/test_event_relay.py tests/test_policy_units.py tests/test_hip_order.py tests/test_kfd_topology.py tests/test_chart_layout.py \
	  tests/test_memory_unit_guards.py tests/test_parity_contract.py tests/test_metrics_exposition.py tests/test_gpu_recovery.py \
	  tests/test_event_matching.py tests/test_relay_protocol.py tests/test_lifecycle_chaos.py tests/test_relay_client.py \
	  -k "not additional_ids and not classification and not bruteforce and not snapshot_reports and not scan_reads_only and not another_namespace and not without_client_id and not partitions_read and not parser_edge and not hosted and not event_types_parse"
	@if ls build/asan-logs/* >/dev/null 2>&1; then cat build/asan-logs/*; exit 1; fi

# Line coverage of native/src from the unit, stress and CPU end-to-end suites.
coverage:
	$(PY) tools/coverage.py --out build/coverage.txt

# -Wall -Wextra as errors over the whole native tree, Python byte-compilation,
# and clang-format / pyflakes when the machine has them.
# Clang static analyzer over native/src, native/mock and native/tools; fails
# on any warning not judged harmless in tools/analyze.py (KNOWN).
analyze:
	$(PY) tools/analyze.py

lint:
	cmake -S native -B build/lint -G Ninja -DCMAKE_BUILD_TYPE=Release "-DCMAKE_CXX_FLAGS=-Werror -Wshadow" >/dev/null
	ninja -C build/lint -j$(JOBS)
	$(PY) -m compileall -q k8s_gpu_sharing_plugin_amd tests tools bench.py __graft_entry__.py
	@command -v clang-format >/dev/null && find native -name '*.cc' -o -name '*.h' | xargs clang-format --dry-run -Werror || echo "clang-format not installed; skipped"
	@$(PY) -m pyflakes k8s_gpu_sharing_plugin_amd tests 2>/dev/null || echo "pyflakes not installed; skipped"

image:
	$(MAKE) -f deployments/container/Makefile build-ubuntu

# Without a container engine: assemble the runtime/validation stages of
# Dockerfile.ubuntu as root filesystems and run the daemon in them (chrooted,
# unprivileged user namespace), against a stub kubelet.
image-rootfs: build
	$(PY) -c "from k8s_gpu_sharing_plugin_amd.utils import build; build.build_image_tree()"
	$(PY) -m pytest -q tests/test_image_rootfs.py tests/test_image_deps.py

clean:
	rm -rf build
