"""The bounded model check of the health state machine (native/tests/health_model.cc).

Every sequence of up to N steps over 16 events -- resets, polls answered or
not, ECC rising or reset, relay drops / restarts / lost events (in-process:
failing event waits, an unplaceable reset), SIGHUP, container restart, drain,
undrain, return-to-service, the hold passing -- in both event layouts, against
a reference model (invariants I1-I10 in the file). `make test-native` runs
depth 6; here depth 5 keeps the CPU suite quick. The sequences it found
broken are pinned below as replays.

Reference: the reference's health loop has no recovery and no test
(/root/reference/cmd/nvidia-device-plugin/nvidia.go:181-269).
"""

import re
import subprocess

import pytest

from k8s_gpu_sharing_plugin_amd import binary

MODEL = binary("adp_health_model")


def test_every_sequence_of_five_steps_keeps_the_invariants():
    r = subprocess.run([MODEL, "--depth", "5", "--jobs", "4"], capture_output=True, text=True, timeout=600)
    m = re.search(r"all (\d+) sequences of 1\.\.5 steps covered by (\d+) distinct states .* (\d+) violation", r.stdout)
    assert r.returncode == 0 and m, r.stdout[-3000:]
    assert int(m.group(1)) == 2 * sum(16 ** i for i in range(1, 6))
    assert int(m.group(2)) > 5000 and int(m.group(3)) == 0, r.stdout


def test_extended_alphabet_every_sequence_of_four_steps():
    """--extended adds GPU 1's resets, an unplaceable GPU_PRE_RESET, the relay
    renewing its registration (in-process: one failing wait), the relay's
    watchdog turning events off and on (relay only), half a hold, GPU 0's
    ECC count turning unreadable and back, and reset events reported by GPU 0's
    second compute partition (GPU 0 is DPX). `make test-native` runs depth 5."""
    r = subprocess.run([MODEL, "--extended", "--depth", "4", "--jobs", "4"], capture_output=True, text=True,
                       timeout=600)
    m = re.search(r"\(extended\), depth 4, 24/25 symbols.* all (\d+) sequences of 1\.\.4 steps covered by (\d+) "
                  r"distinct states .* (\d+) violation", r.stdout)
    assert r.returncode == 0 and m, r.stdout[-3000:]
    assert int(m.group(1)) == sum(24 ** i + 25 ** i for i in range(1, 5))
    assert int(m.group(2)) > 10000 and int(m.group(3)) == 0, r.stdout


def test_random_walks_far_past_the_exhaustive_bound():
    """--random: walks of 60 steps over the extended alphabet, every step
    checked, each probed for liveness at its end (states the depth bound never
    reaches: quarantines over several windows, many relay generations)."""
    r = subprocess.run([MODEL, "--extended", "--random", "400", "--length", "60", "--seed", "3", "--jobs", "4"],
                       capture_output=True, text=True, timeout=600)
    m = re.search(r"400 random walks of 60 steps per layout .*: (\d+) monitor steps.* (\d+) violation", r.stdout)
    assert r.returncode == 0 and m, r.stdout[-3000:]
    assert int(m.group(1)) == 2 * 400 * 60 and int(m.group(2)) == 0, r.stdout


@pytest.mark.parametrize("seq", [
    # an unplaceable GPU_PRE_RESET holds both GPUs; the polled check returns them
    "UNPLACED,POLL_OK,CLOCK_HOLD,POLL_OK",
    # GPU 1 quarantined by its own resets while GPU 0 is untouched; the quiet window ends it
    "PRE1,POST1,PRE1,POST1,CLOCK_HOLD,CLOCK_HOLD,CLOCK_HOLD",
    # an ECC rise while the count could not be read is seen once it can
    "ECC_UNREADABLE,ECC_UP,POLL_OK,ECC_UNREADABLE,POLL_OK",
])
def test_extended_replays(seq):
    r = subprocess.run([MODEL, "--replay", seq], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.count(": ok") == 2, r.stdout + r.stderr


# Found by the model check in round 6 (relay layout): a plugin container
# restarted while its relay connection was down kept a relay cursor up to a
# second old, and the relay's replay re-applied what had been handled:
#  * a GPU_PRE_RESET the operator had since returned held the GPU again;
#  * a GPU_POST_RESET older than an ECC verdict erased the verdict.
# Fix: the cursor is saved when the monitor stops, connected or not, and at
# once after any event that changes a verdict.
# Found by the model check in round 6, once I8 counted resets rather than
# GPU_PRE_RESET events: a PRE that finds the GPU already waiting (every
# partition of a DPX/QPX/CPX GPU reports the same reset) was counted as a new
# reset, so one reset of a CPX GPU quarantined it (end to end:
# test_event_matching.py::test_one_reset_of_a_partitioned_gpu_is_one_reset).
@pytest.mark.parametrize("seq", ["DRAIN,PRE,RETURN,RELAY_DROP,RESTART", "POST,ECC_UP,RELAY_DROP,RESTART,POLL_OK",
                                 "PRE,PRE", "PRE,PRE,POST,PRE", "PRE,POST,PRE"])
def test_pinned_sequences(seq):
    r = subprocess.run([MODEL, "--replay", seq], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok") == 2, r.stdout
