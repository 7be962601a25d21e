"""The certified surface pass's exact redo pass, forced on every path
(nothing exercised the redo pass at the GPU suite's sizes, where
a certificate fails about once in 4 M evaluations).

libptg_certfail.so is libptg.so built with PTG_CERT_FAIL_ALL=1
(csrc/Makefile `certfail`, device/ref_math.h): every rounding certificate of
k_wf_shade<MathFast> fails, so every surface path is listed and shaded again
by k_wf_shade<MathExact> from the same inputs.  Its frames must be the
reference's bit for bit (tests/golden/anim_render_s8.json, the reference's
own whole-image hashes), and the redo tally must cover every surface shade.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT, N

CERTFAIL = os.path.join(os.path.dirname(N.LIB_PATH), "libptg_certfail.so")
FRAMES = [0, 300, 450, 900, 1400, 1750]


def test_certfail_library_built_with_same_abi():
    """The forced-redo test library exists and exports the same C ABI."""
    assert os.path.exists(CERTFAIL), "build it first: __graft_entry__.build() (csrc/Makefile certfail)"

    def syms(p):
        out = subprocess.run(["nm", "-D", "--defined-only", p], stdout=subprocess.PIPE, text=True, check=True).stdout
        return {l.split()[-1] for l in out.splitlines() if l.split() and l.split()[-1].startswith("ptg_")}
    assert syms(CERTFAIL) == syms(N.LIB_PATH)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_forced_redo_pass_bit_identical_to_reference():
    golden = json.load(open(os.path.join(GOLDEN, "anim_render_s8.json")))
    env = dict(os.environ, PTG_LIB=CERTFAIL)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "redo_check.py"), ",".join(map(str, FRAMES))],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["lib"] == "libptg_certfail.so"
    bad = [f for f in FRAMES if out["frames"][str(f)] != golden["frames"][str(f)]]
    assert not bad, "frames differing from the reference with every path redone: %s" % bad
    # the surface shades of the certified pass that evaluated a certified
    # expression were listed and shaded again (a shade that retires before any
    # such evaluation needs no redo); shades (ptg_last_counters[5]) count both
    # passes: first pass = shades - redone
    redo = out["redo"]
    first = out["shades"] - redo["surface"]
    assert redo["surface"] > 0 and redo["sky"] == 0
    assert redo["surface"] <= first and redo["surface"] >= 0.99 * first, (out["shades"], redo)
