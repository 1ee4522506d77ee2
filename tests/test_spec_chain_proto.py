"""Host prototype of the speculative _sum/_avg walk (tools/mb/spec_chain.c,
DESIGN.md section 5): 64 'lanes' x W steps per superstep from estimated
starts, shifted onto the true chain and checked step by step, restarting at
the first failing step.  The prototype must reproduce the sequential gk:53-54
chain bit for bit for every value distribution it generates (lognormal,
small integers, descending, Pareto, signed e^+-50 magnitudes, zeros of both
signs), at W = 16 (the kernel's GK_SPEC_W) and 32.  CPU only."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "mb", "spec_chain.c")


@pytest.fixture(scope="module")
def proto(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("spec") / "spec_chain")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", SRC, "-o", exe, "-lm"], check=True)
    return exe


@pytest.mark.parametrize("w", [16, 32])
@pytest.mark.parametrize("dist", [0, 1, 2, 3, 4, 5])
def test_spec_walk_is_bit_exact(proto, w, dist):
    out = subprocess.run([proto, "200000", str(w), str(dist)], check=True, capture_output=True, text=True).stdout
    m = re.search(r"rounds/superstep: avg ([0-9.]+) sum ([0-9.]+)\s+exact avg (\d) sum (\d)", out)
    assert m, out
    assert m.group(3) == "1" and m.group(4) == "1", out
    assert float(m.group(1)) >= 1.0 and float(m.group(2)) >= 1.0
