"""The host library's tests under AddressSanitizer + UndefinedBehaviorSanitizer
(`-fsanitize=address` for the host sampler).

tools/asan_host_tests.sh builds host/*.cpp (sampler, CPython-set emulation,
graph builder, extend_nodes, pack writers) with -fsanitize=address,undefined
as a host-only library and reruns tests/test_host_sampler.py and
tests/test_unsup_native.py (CPU part) against it in a child process with
libasan preloaded; any sanitizer report aborts that process and fails this
test.  (Kernels and the GPU runner are not covered: GPU ASan is unavailable
on the pool.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _have_asan():
    if not shutil.which("gcc"):
        return False
    lib = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    return os.path.isabs(lib) and os.path.exists(lib)


@pytest.mark.skipif(not _have_asan(), reason="gcc without libasan")
def test_host_library_under_asan_ubsan():
    env = dict(os.environ)
    env.pop("GS_HOST_ASAN_LIB", None)
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_host_tests.sh")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=900)
    tail = (p.stdout + p.stderr)[-4000:]
    assert p.returncode == 0, tail
    assert " passed" in p.stdout and "failed" not in p.stdout, tail
