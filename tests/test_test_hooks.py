"""Fault-injection hooks are compiled out of what ships (round-6 review item 4).

The development tree honours ADP_DEBUG_* variables (the relay refusing or
dropping events, widened race windows in the supervisor) so the CPU suites can
inject faults. The image stages build with -DADP_TEST_HOOKS=OFF: the shipped
daemon does not contain the variable names at all, so a stray variable (a
chart's extraEnv) cannot disable reset handling in production. build/image is
that build, made with the Dockerfiles' cmake line (utils/build.py
build_image_tree; `make image-rootfs` and the assembled-image tests use it).
"""

import os
import re

from k8s_gpu_sharing_plugin_amd import DAEMON, REPO_ROOT
from k8s_gpu_sharing_plugin_amd.utils import build, image

from test_event_relay import RelayNode

HOOKS = [b"ADP_DEBUG_RELAY_REFUSE_EVENT", b"ADP_DEBUG_RELAY_DROP_ON", b"ADP_DEBUG_PUBLISH_DELAY_MS",
         b"ADP_DEBUG_SOCKET_RECHECK_MS"]


def test_image_stages_build_without_the_hooks():
    for dist in ("ubuntu", "ubi9"):
        text = open(os.path.join(REPO_ROOT, "deployments", "container", f"Dockerfile.{dist}")).read()
        cmake = re.search(r"cmake -S native -B /build[^&]*", text.replace("\\\n", " ")).group(0)
        assert "-DADP_TEST_HOOKS=OFF" in cmake, (dist, cmake)
    assert build.IMAGE_CMAKE == ["-DADP_TEST_HOOKS=OFF"]


def test_shipped_daemon_contains_no_hook():
    image.ensure_image_tree()
    shipped = open(image.IMAGE_DAEMON, "rb").read()
    dev = open(DAEMON, "rb").read()
    for h in HOOKS:
        assert h not in shipped, h
        assert h in dev, h  # the development build keeps them (the fault-injection tests need them)
    assert b"ADP_DEBUG_" not in shipped


def test_hook_variables_change_nothing_in_the_shipped_relay(scratch):
    """The shipped relay with every relay hook set to match the reset: the
    GPU_PRE_RESET still reaches the daemon (the dev build would refuse it, and
    drop the daemon's connection, tests/test_event_relay.py)."""
    image.ensure_image_tree()
    n = RelayNode(scratch, relay_env={"ADP_DEBUG_RELAY_REFUSE_EVENT": "type=3", "ADP_DEBUG_RELAY_DROP_ON": "type=3"},
                  relay_launch=lambda argv: [image.IMAGE_DAEMON, *argv[1:]])
    try:
        n.d.wait_log("events on through the relay")
        n.inject("1 3 a reset the hooks would have refused")
        assert n.wait_health(["Healthy", "Unhealthy"]) == ["Healthy", "Unhealthy"]
        rlog = n.relay.log()
        assert "event dropped" not in rlog and "every daemon connection dropped" not in rlog
        assert n.relay.proc.args[0] == image.IMAGE_DAEMON
    finally:
        n.stop()
