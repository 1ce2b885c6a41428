"""CPU: scripts/traffic_json.py -- the per-phase HBM bytes bench.py puts in `roofline.traffic` -- still
recognises the step's kernels.  Its phase table matches exact kernel names (template arguments
included), so a kernel whose name changes (a new template parameter, say) silently drops its phase
from the traffic file; this test takes the committed full run measured on the current sources and
checks every bench phase against its rocprofv3 statistics and traffic file."""
import csv
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import traffic_json as tj  # noqa: E402

# the headline step's phases (bench.py's live brackets, f32split)
STEP_PHASES = ("stft_mel", "db_dct", "conv1_stats", "conv2_fwd", "bn2_pool", "conv3_fwd", "head_fwd", "head_mid",
               "head_dgrad", "head_bwd", "conv3_wgrad", "conv3_dgrad", "bn2_bwd", "conv2_wgrad", "conv2_dgrad",
               "conv1_bwd_wgrad")


def current_run():
    """profiles/<tag> of the full run measured on THESE sources (its traffic file's csrc_sha1 equals
    theirs, as bench.py requires); skipped while the sources have no such run yet."""
    sha = tj.csrc_sha1(ROOT)
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        tag = f[: -len("_traffic.json")]
        if json.load(open(f)).get("csrc_sha1") == sha and os.path.exists(tag + "_kernel_stats.csv"):
            return tag
    pytest.skip("no full run on these sources yet (scripts/round_full.sh + scripts/collect_round.sh)")


def test_phase_table_names_the_profiled_kernels():
    tag = current_run()
    names = {tj.kernel_key(r["Name"]) for r in csv.DictReader(open(tag + "_kernel_stats.csv"))}
    missing = [ph for ph in STEP_PHASES if not any(k in names for k, _ in tj.PHASE_KERNELS[ph])]
    assert not missing, f"{os.path.basename(tag)}: no PHASE_KERNELS candidate for {missing}"


def test_traffic_file_covers_every_phase():
    got = json.load(open(current_run() + "_traffic.json"))
    assert set(STEP_PHASES) <= set(got["bytes_per_launch"]), sorted(set(STEP_PHASES) - set(got["bytes_per_launch"]))
