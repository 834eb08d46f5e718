"""The C ABI from plain C, and the host library under AddressSanitizer +
UndefinedBehaviorSanitizer (sanitizers on the C++ host
library; device code is not instrumented — GPU ASan is unavailable on this
pool).

* tests/native/abi_c: the receiver round of media_client.rs:223-321 written
  in C against include/quack_hip.h (how the Rust FFI binds it), host mode
  here, device mode under -m gpu;
* the same program and tests/test_host_abi.py + tests/test_receiver.py
  (host paths) against libquack_hip_asan.so (sidekick_amd/csrc Makefile
  target `asan`: every host object with -fsanitize=address,undefined), with
  the clang ASan runtime preloaded into Python;
* field.h's native checks under the same sanitizers."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
CLANG = "/opt/rocm/lib/llvm/bin/clang"


def _make(*targets):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sidekick_amd", "csrc"), *targets], check=True,
                   timeout=900)


@pytest.fixture(scope="module")
def native():
    _make("all", "asan")
    subprocess.run(["make", "-s", "-C", NATIVE], check=True, timeout=300)
    return NATIVE


def _asan_runtime():
    return subprocess.run([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True,
                          check=True).stdout.strip()


def test_abi_c_host(native):
    r = subprocess.run([os.path.join(native, "abi_c"), "host"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "4 missing recovered" in r.stdout


def test_abi_c_host_asan(native):
    r = subprocess.run([os.path.join(native, "abi_c_asan"), "host"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr


def test_field_checks_asan(native):
    r = subprocess.run([os.path.join(native, "field_check_asan"), "check"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "0 failures" in r.stdout, r.stdout + r.stderr


def test_host_abi_suite_under_asan(native):
    env = dict(os.environ, LD_PRELOAD=_asan_runtime(), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               QK_LIB_PATH=os.path.join(ROOT, "sidekick_amd", "libquack_hip_asan.so"))
    probe = ("import ctypes, sidekick_amd._lib as L; L.lib(); "
             "assert L.LIB_PATH.endswith('_asan.so'); ctypes.CDLL(None).__asan_init; print('asan-loaded')")
    r = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 0 and "asan-loaded" in r.stdout, r.stdout + r.stderr
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        "tests/test_host_abi.py", "tests/test_receiver.py"], capture_output=True, text=True,
                       timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout


@pytest.mark.gpu
def test_abi_c_device():
    """The C round with the sender's batch encode and the log's root test on
    the GPU (qk_u32_encode_host, qk_u32_decode_device)."""
    exe = os.path.join(NATIVE, "abi_c")
    assert os.path.exists(exe), "build tests/native first (__graft_entry__.build())"
    r = subprocess.run([exe, "device"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_c device ok" in r.stdout


def test_abi_failure_paths_host_no_leaks(native):
    """tests/native/abi_fail: every host error path of the ABI 3000 times,
    plain and under ASan with the leak checker on."""
    r = subprocess.run([os.path.join(native, "abi_fail"), "host"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "abi_fail host ok" in r.stdout, r.stdout + r.stderr
    r = subprocess.run([os.path.join(native, "abi_fail_asan"), "host", "1000"], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    assert r.returncode == 0 and "abi_fail host ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
def test_abi_failure_paths_device_no_growth():
    """The device entry points' failures (early argument checks and late
    capacity / undecodable returns after kernels ran) 300 times on one
    context: every status as documented, device memory flat."""
    exe = os.path.join(NATIVE, "abi_fail")
    assert os.path.exists(exe), "build tests/native first (__graft_entry__.build())"
    r = subprocess.run([exe, "device", "300"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "abi_fail device ok" in r.stdout, r.stdout + r.stderr
