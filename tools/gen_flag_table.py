"""Renders the daemon's flag table (from `amdgpu-device-plugin --help`) as Markdown.

  python tools/gen_flag_table.py > /tmp/flags.md
  python tools/gen_flag_table.py --update docs/USER_GUIDE.md   # rewrite the table in place
Used to keep docs/USER_GUIDE.md in step with the binary (tests/test_docs.py).
"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_sharing_plugin_amd import DAEMON  # noqa: E402


def flags():
    text = subprocess.run([DAEMON, "--help"], capture_output=True, text=True, check=True).stdout
    out = []
    lines = text.splitlines()
    for i, line in enumerate(lines):
        m = re.match(r"^  --([a-z0-9-]+)  \(env (\w+)(?:, file (flags\.\w+))?, default (.*)\)$", line)
        if m:
            out.append({"flag": m.group(1), "env": m.group(2), "file": m.group(3) or "", "default": m.group(4),
                        "help": lines[i + 1].strip()})
    return out


def table():
    rows = ["| flag | env | config file | default | meaning |", "|---|---|---|---|---|"]
    for f in flags():
        file_key = f"`{f['file']}`" if f["file"] else ""
        help_text = f["help"].replace("|", "\\|")
        rows.append(f"| `--{f['flag']}` | `{f['env']}` | {file_key} | `{f['default']}` | {help_text} |")
    return "\n".join(rows) + "\n"


def update(path):
    """Replaces the first flag table (header row + `--flag` rows) of `path`."""
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.startswith("| flag |"))
    end = start + 2
    while end < len(lines) and lines[end].startswith("| `--"):
        end += 1
    lines[start:end] = table().rstrip("\n").split("\n")
    open(path, "w").write("\n".join(lines))


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--update":
        update(sys.argv[2])
    else:
        sys.stdout.write(table())
