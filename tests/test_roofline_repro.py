"""The bench line's roofline numbers follow from the committed profiles
alone (tools/roofline_repro.py): PMC counts per launch over the measured
ceilings, divided by the launch time; the rocprof trace's launch time agrees
with the bench's HIP-event time."""
import glob
import os
import subprocess
import sys

from conftest import ROOT


def test_newest_bench_line_roofline_reproduces():
    lines = glob.glob(os.path.join(ROOT, "profiles", "*", "bench_line.json"))
    assert lines
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_repro.py")], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=60)
    assert r.returncode == 0 and "reproduced" in r.stdout, r.stdout
