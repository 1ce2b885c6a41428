"""CPU: the plain-C host of the C ABI (examples/c_host/abd_c_host.c) builds against include/abd.h and
resolves libabd.so through its run path; argument errors are reported before any HIP call."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "c_host", "abd_c_host")

pytestmark = pytest.mark.skipif(not os.access(EXE, os.X_OK), reason="not built (make -C audio-backdoor-attack_amd)")


def test_c_host_links_libabd_in_tree():
    ldd = subprocess.run(["ldd", EXE], capture_output=True, text=True, check=True).stdout
    line = [ln for ln in ldd.splitlines() if "libabd.so" in ln]
    assert line and os.path.realpath(line[0].split("=>")[1].split("(")[0].strip()) == \
        os.path.realpath(os.path.join(ROOT, "audio-backdoor-attack_amd", "libabd.so"))


def test_c_host_argument_errors():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and "usage:" in r.stderr
    r = subprocess.run([EXE, "/nonexistent", "0", "35"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and "B >= 1 and K >= 2 required" in r.stderr
