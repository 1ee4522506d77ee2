"""Build-level invariants of the HIP kernels (no GPU needed: hipcc
cross-compiles for gfx950 here)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sketches-py_amd", "csrc")


@pytest.fixture(scope="module")
def resource_report(tmp_path_factory):
    out = tmp_path_factory.mktemp("res") / "k.o"
    r = subprocess.run(
        ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-Wno-unused-result", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
         "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(CSRC, "gk_kernels.hip"), "-o", str(out)],
        capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    kernels = {}
    cur = None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        m = re.search(r"remark:\s+(.+?): (\d+) \[", line)
        if cur and m:
            kernels[cur][m.group(1).strip()] = int(m.group(2))
    return kernels


@pytest.fixture(scope="module")
def small_isa(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "k.s"
    r = subprocess.run(
        ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-Wno-unused-result", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, "--cuda-device-only", "-S",
         os.path.join(CSRC, "gk_kernels.hip"), "-o", str(out)],
        capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    text = open(out).read()
    bodies = {}
    for m in re.finditer(r"^(_Z14k_ingest_small\w+):", text, re.M):
        end = text.index("s_endpgm", m.end())
        bodies[m.group(1)] = text[m.end():end]
    return bodies


def test_fast_class_has_no_scratch(resource_report, small_isa):
    """The small class runs nearly every stream: no scratch traffic in the
    per-flush path.  The allocator folds a few loop-invariant per-lane LDS /
    global addresses into scratch: stored once at kernel entry, reloaded once
    per stream (end-of-stream pending copy, the empty-table first flush).
    Keeping them in registers instead (e.g. re-reading the gap info at emit)
    measured 1-2% slower (profiles/archive/r01t_ab_regpressure_REJECTED.txt), so the
    bound is on the count: a spill inside the flush loops adds many more.
    The stats role (fused_stats_role, run by a few waves before they join the
    hand-out) adds one more folded value (48 bytes, 11 scratch instructions
    at most); the ingest-only launch measured the same with and without it
    (GK_FUSED_STATS=0 rows of profiles/archive/r01z_ab_fused_stats.txt).
    The VPL=1 instance (P <= 64) carries more since the DPP lane exchanges
    (profiles/r02k_dpp_exchanges_sq.txt: one 4-byte reload per flush) and the
    paced stats role (per-batch reloads of its part bounds,
    profiles/r02y_stats_pacing_ab.txt).
    Since v18 the stats role is a template flag (4 instances: VPL 1/2, with
    and without the role); the bench's instance (VPL=2 with the role, 5.90 ms
    per cfg3 launch at 23 scratch instructions) sets the bounds."""
    fast = {k: v for k, v in resource_report.items() if k.startswith("_Z14k_ingest_small")}
    assert len(fast) == 4
    for k, v in fast.items():
        assert v.get("ScratchSize [bytes/lane]", 0) <= 64, (k, v)
    for name, body in small_isa.items():
        ops = re.findall(r"^\s*(scratch_\w+)", body, re.M)
        assert len(ops) <= 24, (name, ops)


def test_no_inline_asm_memory_ops():
    """Inline-asm loads were rejected: the compiler may copy an asm output
    register before the load lands (tools/check_async_loads.py found such
    copies).  Memory operations in the kernels stay compiler-visible."""
    src = open(os.path.join(CSRC, "gk_kernels.hip")).read()
    for m in re.finditer(r'asm\s+volatile\s*\(\s*"([^"]*)"', src):
        assert "load" not in m.group(1) and "store" not in m.group(1), m.group(1)


def test_fast_class_occupancy(resource_report):
    k = [v for n, v in resource_report.items() if n.startswith("_Z14k_ingest_smallILi2E")][0]
    assert k["Occupancy [waves/SIMD]"] >= 4
    assert k["LDS Size [bytes/block]"] <= 9 * 1024
