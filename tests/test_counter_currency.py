"""CPU test that the committed counter summaries describe the kernels the final build runs.

bench.py divides live HIP-event times by the per-launch counters of profiles/sq_issue.json (the `issue`
block) and reports profiles/pmc_traffic.json's HBM bytes as `traffic`. Both must come from one profiling
session of the final build, taken after the round's last kept kernel change, and name the k_bake
instance(s) the bench line ran (fmgi_last_bake_kernel, `roofline.counters.kernel`):
  - profiles/r06/README.md names the last kept kernel change, the counter session and the final bench session
    in three marker lines;
  - every config's summaries cite the counter session, which is not older than the last kept change;
  - the final bench session (same build, after the summaries were committed) reports, per config, the kernel
    instance the summaries name, and the bench matched them (`issue_matches_kernel`, `traffic_matches_kernel`).
"""
import json
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "profiles")
CONFIGS = ("box200", "example", "box2000")


def _markers():
    text = open(os.path.join(PROF, "r06", "README.md")).read()
    last = re.search(r"^last kept kernel change: s(\d+)", text, re.M)
    sess = re.search(r"^counter session: s(\d+)", text, re.M)
    final = re.search(r"^final bench session: s(\d+)", text, re.M)
    assert last and sess and final, "profiles/r06/README.md lacks its marker lines"
    return int(last.group(1)), int(sess.group(1)), int(final.group(1))


def _session_of(source):
    m = re.match(r"profiles/r06/s(\d+)", source)
    assert m, f"counter source {source!r} is not a round-6 session"
    return int(m.group(1))


def test_counter_session_postdates_the_last_kept_change():
    last, sess, final = _markers()
    assert final >= sess >= last, (final, sess, last)
    assert os.path.isdir(os.path.join(PROF, "r06", f"s{sess}")) and os.path.isdir(os.path.join(PROF, "r06", f"s{final}"))


@pytest.mark.parametrize("config", CONFIGS)
def test_summaries_name_the_bench_instance(config):
    _, sess, final = _markers()
    sq = json.load(open(os.path.join(PROF, "sq_issue.json")))[config]
    pmc = json.load(open(os.path.join(PROF, "pmc_traffic.json")))[config]
    assert _session_of(sq["source"]) == sess and _session_of(pmc["source"]) == sess
    assert sq["kernel"] == pmc["kernel"] and sq["kernel"].startswith("void (anonymous namespace)::k_bake<")
    bench = os.path.join(PROF, "r06", f"s{final}", f"bench_{config}.log")
    line = [l for l in open(bench) if l.startswith("{")]
    assert len(line) == 1, bench
    out = json.loads(line[0])
    c = out["roofline"]["counters"]
    assert c["kernel"] == sq["kernel"], (c["kernel"], sq["kernel"])
    assert c["issue_matches_kernel"] and c["traffic_matches_kernel"]
    assert out["roofline"]["issue"] is not None and out["roofline"]["traffic"] == pytest.approx(
        pmc["hbm_bytes_per_launch"])
