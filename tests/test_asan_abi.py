"""Host AddressSanitizer run of the C ABI's argument validation (sanitizers).

tools/asan_build.sh compiles api.hip with ``-Xarch_host -fsanitize=address`` (device code
unchanged; GPU sanitizers are not available on this pool) and links
tests/asan/abi_validation.cpp, which calls every entry point of include/itsd.h with each
class of invalid argument and, for a valid descriptor on a machine without a GPU, checks the
clean ITSD_ERR_HIP path. CPU only: no device work is reached.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd")
EXE = os.path.join(ROOT, "build_asan", "abi_validation")


def _stale() -> bool:
    if not os.path.exists(EXE):
        return True
    t = os.path.getmtime(EXE)
    srcs = [os.path.join(PKG, "csrc", f) for f in os.listdir(os.path.join(PKG, "csrc"))]
    srcs += [os.path.join(ROOT, "include", "itsd.h"), os.path.join(ROOT, "tests", "asan", "abi_validation.cpp")]
    return any(os.path.getmtime(s) > t for s in srcs)


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_abi_validation_under_asan():
    if _stale():
        r = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_build.sh")], capture_output=True, text=True,
                           timeout=900)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               HIP_VISIBLE_DEVICES="-1")  # never a device, even on a GPU box
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "ERROR: LeakSanitizer" not in out, out[-4000:]
    assert r.returncode == 0 and "PASSED (0 failures)" in r.stdout, out[-4000:]
