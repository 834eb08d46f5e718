"""Native CPU checks of the shared field arithmetic (sidekick_amd/csrc/field.h):
the t-form step, lazy folds and the p64 helpers against 128-bit arithmetic,
and that the committed wrap-forcing ids really take the rare branch of the
baby-step/giant-step encode (the GPU test that uses them is in
test_gpu_encode.py)."""
import os
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def exe():
    out = os.path.join(tempfile.gettempdir(), f"qk_field_check_{os.getpid()}")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", out, os.path.join(HERE, "native", "field_check.cpp")],
                   check=True)
    yield out
    os.unlink(out)


def test_field_primitives(exe):
    r = subprocess.run([exe, "check"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_wrap_ids_take_the_rare_branch(exe, golden):
    for cfg, ids in golden["bsgs_wrap_ids"].items():
        nb, na = cfg.split("x")
        assert len(ids) >= 4
        for i in ids[:3]:
            r = subprocess.run([exe, "find", nb, na, "1", str(i)], capture_output=True, text=True, timeout=60)
            assert int(r.stdout.split()[0]) == i, (cfg, i)


def test_root_finding_vector_paths_agree_with_scalar():
    """roots.cpp takes one path per CPU (IFMA here and on the GPU box's
    EPYC); tests/native/roots_paths.cpp runs the scalar, AVX-512 and IFMA
    forms of the polynomial squaring (u32, u64) and the u64 row operation on
    the same random and edge inputs and requires identical results."""
    out = os.path.join(tempfile.gettempdir(), f"qk_roots_paths_{os.getpid()}")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(HERE, "..", "include"), "-I",
                    os.path.join(HERE, "..", "sidekick_amd", "csrc"), "-o", out,
                    os.path.join(HERE, "native", "roots_paths.cpp")], check=True)
    try:
        r = subprocess.run([out], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.strip().endswith("ok")
    finally:
        os.unlink(out)
