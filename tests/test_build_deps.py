"""The in-tree build rebuilds on mtime (build.py: `up_to_date`): every file a source includes must be
in DEPS, or an edit to that header alone would leave a stale liblompc_amd.so to be pushed."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))

from lompc_amd import build as B  # noqa: E402


def test_every_quoted_include_is_a_dep():
    deps = {os.path.normpath(os.path.join(B.CSRC, d)) for d in B.DEPS}
    inc = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)
    seen = 0
    for f in sorted(os.listdir(B.CSRC)):
        if not f.endswith((".hip", ".cpp", ".hpp", ".h")):
            continue
        p = os.path.normpath(os.path.join(B.CSRC, f))
        assert p in deps, f"csrc/{f} is not in build.DEPS"
        with open(p) as fh:
            for m in inc.finditer(fh.read()):
                tgt = os.path.normpath(os.path.join(B.CSRC, m.group(1)))
                assert tgt in deps, f'csrc/{f} includes "{m.group(1)}", which is not in build.DEPS'
                seen += 1
    assert seen >= 10
