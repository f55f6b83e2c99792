import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running (multi-process) test")


@pytest.fixture(scope="session", autouse=True)
def native_build():
    """Build the native tree once per session (incremental, seconds when up to date)."""
    from k8s_gpu_sharing_plugin_amd.utils import build
    build.build_native()
    build.build_descriptor()
    return True


@pytest.fixture
def scratch():
    from k8s_gpu_sharing_plugin_amd.utils import harness
    import shutil
    d = harness.scratch_dir("adptest")
    yield d
    shutil.rmtree(d, ignore_errors=True)
    shutil.rmtree(d + ".fixture", ignore_errors=True)
    for suffix in (".daemon.log",):
        try:
            os.unlink(d + suffix)
        except OSError:
            pass


@pytest.fixture
def mock_env(tmp_path, monkeypatch):
    """Point in-process native calls (libadp_capi) at the amdsmi mock with a fixture."""
    from k8s_gpu_sharing_plugin_amd import MOCK_LIB
    from k8s_gpu_sharing_plugin_amd.models import fixtures

    def use(fixture):
        path = fixtures.write(fixture, str(tmp_path))
        monkeypatch.setenv("AMDSMI_MOCK_FIXTURE", path)
        return MOCK_LIB
    return use
