"""The drop-in microbenchmark programs (examples/benchmark_construct.c,
examples/benchmark_decode.c, built into target/release/examples/ where the
reference's figure script runs them) accept the figure's command lines
(figures/fig2_microbenchmarks.py:85-95,134-141,175-183,205-213) and print
SUMMARY lines that its parsers read (:25-69: "avg = <duration>",
"(per-packet): <duration>/packet", Rust Duration formatting)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "target", "release", "examples")


def run(prog, *args):
    r = subprocess.run([os.path.join(BIN, prog), *args], capture_output=True, text=True, timeout=120, cwd=ROOT)
    return r.returncode, r.stdout + r.stderr


def duration_us(v):
    """A Rust Duration Debug string ("34.676µs", "1.2ms", "834ns") in µs."""
    m = re.fullmatch(r"([0-9.]+)(ns|µs|ms|s)", v)
    assert m, v
    return float(m.group(1)) * {"ns": 1e-3, "µs": 1.0, "ms": 1e3, "s": 1e6}[m.group(2)]


def parse(out):
    avg = re.search(r"SUMMARY: num_trials = (\d+), avg_cycles = (\d+), avg = (\S+)", out)
    per = re.search(r"SUMMARY \(per-packet\): (\S+)/packet = (\d+) packets/s = (\d+) cycles/packet", out)
    assert avg and per, out
    return int(avg.group(1)), duration_us(avg.group(3)), duration_us(per.group(1))


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], check=True)


@pytest.mark.parametrize("bits,t", [(32, 10), (32, 80), (64, 30)])
def test_construct_command_line(bits, t):
    args = ["power-sum", "-e", "1000", "--trials", "20", "-t", str(t), "-b", str(bits)]
    if bits == 64:
        args.append("--montgomery")
    rc, out = run("benchmark_construct", *args)
    assert rc == 0, out
    trials, avg_us, per_us = parse(out)
    assert trials == 20 and avg_us > 0
    assert abs(per_us - avg_us / 1000) <= 1e-3 + avg_us / 1000 * 0.01   # per-packet = avg / n (ns granularity)


@pytest.mark.parametrize("bits,d,n", [(32, 10, 300), (32, 300, 300), (64, 20, 300), (64, 10, 40)])
def test_decode_command_lines(bits, d, n):
    args = ["power-sum", "-n", str(n), "--trials", "10", "-d", str(d), "-t", str(d), "-b", str(bits)]
    rc, out = run("benchmark_decode", *args)
    assert rc == 0, out
    trials, avg_us, _ = parse(out)
    assert trials == 10 and avg_us > 0


def test_duration_format_matches_rust_debug():
    # the formats the published logs hold (nsdi24/quack/*): integer and
    # trailing-zero-trimmed fractions per unit
    rc, out = run("benchmark_construct", "power-sum", "-e", "1", "--trials", "3", "-t", "1", "-b", "32")
    assert rc == 0
    v = re.search(r"avg = (\S+)", out).group(1)
    assert re.fullmatch(r"\d+ns|\d+(\.\d*[1-9])?(µs|ms|s)", v), v


@pytest.mark.parametrize("prog,args", [("benchmark_construct", ["power-sum", "-b", "16", "--precompute"]),
                                       ("benchmark_decode", ["power-sum", "-n", "100", "-d", "5", "--factor"]),
                                       ("benchmark_construct", ["strawman1a"])])
def test_out_of_scope_variants_refuse(prog, args):
    rc, out = run(prog, *args)
    assert rc == 2 and ("scope" in out or "only" in out), out


@pytest.mark.gpu
def test_gpu_paths():
    rc, out = run("benchmark_construct", "power-sum", "-e", "100000", "--trials", "5", "-t", "32", "-b", "32", "--gpu")
    assert rc == 0, out
    parse(out)
    rc, out = run("benchmark_construct", "power-sum", "-e", "100000", "--trials", "5", "-t", "80", "-b", "64",
                  "--gpu-resident")
    assert rc == 0, out
    rc, out = run("benchmark_decode", "power-sum", "-n", "100000", "--trials", "5", "-d", "32", "-b", "64", "--gpu")
    assert rc == 0, out
    parse(out)
