"""Host-code sanitizers: the product's text parsers (csrc/ingest.cpp: `scontrol` and
`#SBATCH` text, untrusted input) built with ASan + UBSan (`make -C slurm-bridge-operator_amd
sanitize`) and driven by tools/fuzz_ingest.cpp over mutations of the reference's canned scontrol
text and the C1 fixtures, comparing every result with the oracle's restatement.  Any sanitizer
report or mismatch fails the run."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_ingest_parsers_under_asan_ubsan(tmp_path):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "slurm-bridge-operator_amd"), "sanitize"])
    seeds = [os.path.join(GOLD, f) for f in ("scontrol_show_nodes.txt", "c1_scontrol_show_nodes.txt",
                                             "c1_scontrol_show_partition.txt")]
    vec = json.load(open(os.path.join(GOLD, "reference_vectors.json")))
    for i, case in enumerate(vec["parse_resources"] + vec["parse_partitions_names"]):
        p = tmp_path / f"ref{i}.txt"
        p.write_text(case["in"])
        seeds.append(str(p))
    exe = os.path.join(ROOT, "slurm-bridge-operator_amd", "build", "fuzz_ingest")
    env = {**os.environ, "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"}
    r = subprocess.run([exe, "20000", "11", *seeds], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "0 mismatches" in r.stdout
