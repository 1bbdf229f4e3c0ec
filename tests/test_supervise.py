"""bench.py's supervisor (cuda_knearests_amd/utils/supervise.py), on CPU with fake children: a failed
first attempt on any rank -- an exit code, a hung peer, a missing JSON line -- is re-run by fresh
children on the next path, and rank 0 prints ONE line naming the path that produced it."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from cuda_knearests_amd.utils import REPO
from cuda_knearests_amd.utils.supervise import Attempt, annotate, free_port, json_line, supervise

# the fake timed job: behaviour per (attempt tag, rank) from the environment
CHILD = textwrap.dedent("""
    import json, os, sys, time
    tag, rank = os.environ["KN_T"], int(os.environ.get("RANK", "0"))
    mode = os.environ.get("KN_T_" + tag + "_" + str(rank), "ok")
    print("child", tag, rank, mode, "port", os.environ["MASTER_PORT"], file=sys.stderr, flush=True)
    if mode == "fail":
        print("Traceback: CollectiveError: injected", file=sys.stderr, flush=True)
        sys.exit(3)
    if mode == "hang":
        time.sleep(600)
    if mode == "nojson":
        sys.exit(0)
    if rank == 0:
        print(json.dumps({"metric": "m", "value": 1.0, "tag": tag}), flush=True)
""")


def test_world1_fallback_on_exit_code():
    attempts = [Attempt("native", {"KN_T": "a", "KN_T_a_0": "fail"}, [], 60.0),
                Attempt("torch", {"KN_T": "b"}, [], 60.0)]
    ok, outs = supervise([sys.executable, "-c", CHILD], attempts)
    assert ok == 1 and outs[0].rc == 3 and outs[1].rc == 0
    line = annotate(outs[1].line, attempts, ok, outs)
    assert line["dist_path"] == "torch" and line["tag"] == "b" and line["first_attempt_rc"] == 3
    assert any("CollectiveError" in s for s in line["failed_attempts"][0]["stderr_tail"])


def test_world1_missing_json_line_fails_the_attempt():
    attempts = [Attempt("native", {"KN_T": "a", "KN_T_a_0": "nojson"}, [], 60.0),
                Attempt("torch", {"KN_T": "b"}, [], 60.0)]
    ok, outs = supervise([sys.executable, "-c", CHILD], attempts)
    assert ok == 1
    assert annotate(outs[1].line, attempts, ok, outs)["first_attempt_rc"] == "no JSON line"


def test_world1_first_attempt_ok():
    attempts = [Attempt("native", {"KN_T": "a"}, [], 60.0), Attempt("torch", {"KN_T": "b"}, [], 60.0)]
    ok, outs = supervise([sys.executable, "-c", CHILD], attempts)
    assert ok == 0 and len(outs) == 1
    line = annotate(outs[0].line, attempts, ok, outs)
    assert line["dist_path"] == "native" and line["first_attempt_rc"] == 0 and "failed_attempts" not in line


PARENT = textwrap.dedent("""
    import json, sys
    sys.path.insert(0, {repo!r})
    from cuda_knearests_amd.utils.supervise import Attempt, annotate, make_store, supervise
    import os
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    attempts = [Attempt("native", {{"KN_T": "a"}}, [], 60.0), Attempt("torch", {{"KN_T": "b"}}, [], 60.0)]
    ok, outs = supervise([sys.executable, "-c", {child!r}], attempts, rank, world, make_store(rank, world))
    if rank == 0 and ok >= 0:
        print(json.dumps(annotate(outs[ok].line, attempts, ok, outs)), flush=True)
    sys.exit(0 if ok >= 0 else 1)
""")


@pytest.mark.parametrize("case", ["peer_fails_rank0_hangs", "rank0_fails", "all_ok"])
def test_world2_parents_agree(case):
    """Two parent ranks over their own TCP store (rank 0 hosts it, as without torchrun's agent
    store). A failing rank 1 while rank 0's child hangs: rank 0's parent kills its child at once (not
    at the attempt's timeout) and both run the second attempt."""
    port = free_port()
    modes = {"peer_fails_rank0_hangs": {"KN_T_a_1": "fail", "KN_T_a_0": "hang"},
             "rank0_fails": {"KN_T_a_0": "fail"}, "all_ok": {}}[case]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **modes)
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        procs.append(subprocess.Popen([sys.executable, "-c", PARENT.format(repo=str(REPO), child=CHILD)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    assert outs[1][0].strip() == ""  # only rank 0 prints
    lines = [ln for ln in outs[0][0].splitlines() if ln.strip()]
    assert len(lines) == 1
    line = json.loads(lines[0])
    if case == "all_ok":
        assert line["dist_path"] == "native" and line["tag"] == "a"
        return
    assert line["dist_path"] == "torch" and line["tag"] == "b"
    fa = line["failed_attempts"][0]
    assert fa["failed_rank"] == (1 if case == "peer_fails_rank0_hangs" else 0) and fa["rc"] == 3
    assert [x["rank"] for x in fa["failed_ranks"]] == [fa["failed_rank"]]
    assert line["first_attempt_rc"] == 3 and len(fa["rank_rcs"]) == 2
    assert any("CollectiveError" in s for s in fa["stderr_tail"])


def test_json_line_picks_the_metric_line():
    assert json_line('noise\n{"a": 1}\n{"metric": "x", "value": 2}\ntrailing\n')["value"] == 2
    assert json_line("no json here") is None


def test_bench_supervised_single_gpu_path_without_gpu():
    """bench.py on a host without a GPU: both 1-GPU attempts fail (no HIP device), the parent
    reports it and exits non-zero without printing a line (no number is ever invented)."""
    env = dict(os.environ, KN_BENCH_ATTEMPT_S="120")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--steps", "1", "--warmup", "0", "--n", "1000"],
                       capture_output=True, text=True, timeout=600, env=env)
    if r.returncode == 0:
        pytest.skip("a GPU is visible")
    assert r.stdout.strip() == ""
    assert "attempt pipelined failed" in r.stderr and "every attempt failed" in r.stderr
