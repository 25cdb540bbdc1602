"""The reference-side binding compiles against the reference's headers.

integration/check_shim.sh stages integration/esa_linsmax.{c,h} as
src/match/ and the reference's src/tools/gt_repfind.c with
integration/gt_repfind_smax.patch applied, and compiles both with gcc
(-Werror) against /root/reference/src and this repo's include/.  The
reference tree exists only in the build container: skipped elsewhere.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "src", "tools", "gt_repfind.c")),
                    reason="reference tree not present")
def test_shim_and_runner_patch_compile_against_reference():
    r = subprocess.run(["sh", os.path.join(ROOT, "integration", "check_shim.sh"), REF],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_shim_binds_only_declared_entry_points():
    """Every gt_smax_/gt_maxpairs_ function the shim calls is declared in
    include/ (and therefore exported, tests/test_capi.py)."""
    import re
    import genometools_smax_amd as G
    with open(os.path.join(ROOT, "integration", "esa_linsmax.c")) as fh:
        src = fh.read()
    called = set(re.findall(r"\b(gt_(?:smax|maxpairs)_hip_\w+)\s*\(", src))
    assert called == {"gt_smax_hip_enumerate", "gt_maxpairs_hip_enumerate"}
    assert called <= set(G.exported_symbols())


SHIM_EXEC = os.path.join(ROOT, "integration", "exec_test", "_build", "shim_exec")


@pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "src", "match", "sarr-def.h")),
                    reason="reference tree not present")
def test_shim_links_into_an_executable():
    """integration/exec_test/build.sh: the shim compiled against the
    reference's headers, linked with test doubles of the reader and with
    libgtsmax_hip.so (tests/test_shim_exec_gpu.py runs it on the GPU)."""
    r = subprocess.run(["sh", os.path.join(ROOT, "integration", "exec_test", "build.sh"), REF],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert os.access(SHIM_EXEC, os.X_OK)


@pytest.mark.skipif(not os.path.isfile(SHIM_EXEC), reason="shim executable not built")
def test_shim_reports_reader_errors_through_gterror(tmp_path):
    """A missing index fails in the reader (no GPU call): exit 1 and the
    reader's message, copied through GtError as gt_callenummaxpairs does."""
    r = subprocess.run([SHIM_EXEC, str(tmp_path / "none"), "8", "smax"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 1
    assert "cannot open file" in r.stderr and r.stdout == ""
