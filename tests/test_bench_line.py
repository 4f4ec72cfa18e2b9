"""bench.py's JSON line on the GPU (a reduced block count): the driver's contract keys, the
dominant kernel's roofline beside both halves, and the self-check of the round trip."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_is_verified_and_complete():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--blocks", "2048", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", "--host-steps", "0"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in line, key
    assert line["verified"] is True
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["value"] > 0
    rf = line["roofline"]
    assert rf["dominant_of_step"] in ("encode", "decode")
    half = line["roofline_" + rf["dominant_of_step"]]
    assert rf["achieved"] == half["achieved"] and rf["kernel"] == half["kernel"]
    ms = line["kernels_ms"]
    assert rf["dominant_of_step"] == ("decode" if ms["decode"] > ms["encode"] else "encode")
    assert 0 < rf["frac"] < 1.2


def test_two_ranks_sharing_one_gpu():
    """The N-rank path of bench.py on a one-GPU box (--share-gpu: both ranks on cuda:0, gloo for
    the barrier and the reductions): weak-scaled block ranges, max-over-ranks timing, every
    rank's round trip verified, the CPU baseline on rank 0 only, one line marked as a rehearsal."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu",
                        "--blocks", "2048", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--host-steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["verified"] is True and "rehearsal" in line
    assert line["config"]["blocks_total"] == 4096 and line["config"]["blocks_per_gpu"] == 2048
    assert line["host_resident"]["value"] > 0 and line["value"] > 0
