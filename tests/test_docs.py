"""Docs stay in step with the binary: every flag of `--help` is documented."""

import os

from k8s_gpu_sharing_plugin_amd import REPO_ROOT


def test_user_guide_documents_every_flag():
    import sys
    sys.path.insert(0, os.path.join(REPO_ROOT, "tools"))
    import gen_flag_table
    guide = open(os.path.join(REPO_ROOT, "docs", "USER_GUIDE.md")).read()
    flags = gen_flag_table.flags()
    assert len(flags) >= 20
    for f in flags:
        assert f"`--{f['flag']}`" in guide and f"`{f['env']}`" in guide, f
    assert gen_flag_table.table() in guide, "regenerate the table: python tools/gen_flag_table.py"


def test_docs_link_targets_exist():
    import re
    for doc in ("README.md", "docs/USER_GUIDE.md", "docs/SHARING_TUTORIAL.md", "docs/PERF.md", "docs/PARITY.md",
                "docs/ARCHITECTURE.md"):
        text = open(os.path.join(REPO_ROOT, doc)).read()
        for path in set(re.findall(r"`((?:examples|deployments|native|tools|profiles|docs)/[\w./-]+)`", text)):
            path = path.rstrip(".")
            if "*" in path or "{" in path or path.endswith("_") or "nvidia" in path:
                continue
            assert os.path.exists(os.path.join(REPO_ROOT, path)), f"{doc}: {path}"


def test_metrics_reference_lists_every_exported_family():
    """docs/USER_GUIDE.md "Metrics reference" names every metric family the
    daemon exports, and nothing it does not."""
    import glob
    import re
    src = "".join(open(f).read() for f in glob.glob(os.path.join(REPO_ROOT, "native", "src", "*", "*.cc")))
    exported = {n for n in re.findall(r"amdgpu_dp_[a-z0-9_]+", src) if not n.endswith(("_bucket", "_sum", "_count"))}
    guide = open(os.path.join(REPO_ROOT, "docs", "USER_GUIDE.md")).read()
    section = guide.split("### Metrics reference", 1)[1].split("\n## ", 1)[0]
    documented = set(re.findall(r"^\| `(amdgpu_dp_[a-z0-9_]+)`", section, re.M))
    assert documented == exported, (sorted(exported - documented), sorted(documented - exported))
