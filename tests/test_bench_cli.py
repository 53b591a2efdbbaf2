"""CPU tests of bench.py's multi-rank launcher (the path the 1/2/4/8-GPU scaling run takes).

``--cpu-plumbing`` swaps the forward for a stand-in step so the launcher, the gloo all_gather of
ScenePlanner, the barrier / max-over-ranks timing and the rank-0 JSON run here without a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=timeout, cwd=ROOT)


def test_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--cpu-plumbing", "--steps", "3", "--warmup", "1", "--batch", "4"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2
    assert j["config"]["global_batch"] == 8
    assert j["config"]["gathered_rows"] == 8
    assert j["config"]["ranks_seen"] == [0, 1]
    # the bench's own gather check (bench.gather_slices_ok): every rank's slice equals its local step, agreed by MIN
    assert j["gather_check"] == {"gathered_rows": 8, "every_rank_slice_equals_local": True}
    assert j["value"] > 0 and j["scaling"] == "weak"


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "1", "--cpu-plumbing", "--steps", "1", "--warmup", "0"],
             env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "disagrees" in r.stderr


def test_single_rank_plumbing():
    r = _run(["--cpu-plumbing", "--steps", "2", "--warmup", "0", "--batch", "2"])
    assert r.returncode == 0, r.stderr
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["n_gpus"] == 1 and j["config"]["global_batch"] == 2


def test_gpus2_three_lanes_in_flight_plumbing():
    """bench.py's lane path at --in-flight 3 over gloo with two ranks: the bench's own LaneSteps drives an
    InFlightPlanner of three stand-in lanes (its real round-robin), every step all-gathers on its lane's stream, and
    the bench's gather check holds. Each step's issue lands on the next lane in order, each lane's stream sees
    [event, forward, event] per step in step order, and the last gather holds one step's rows from both ranks
    (the ranks issue their collectives in the same step order, so lanes cannot cross-match the ring)."""
    r = _run(["--gpus", "2", "--cpu-plumbing", "--in-flight", "3", "--steps", "7", "--warmup", "2", "--batch", "3"])
    assert r.returncode == 0, r.stderr
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert j["config"]["in_flight"] == 3 and j["config"]["ranks_seen"] == [0, 1]
    lanes = j["lanes"]
    assert lanes["issue_order"] == [i % 3 for i in range(9)]
    assert lanes["each_step_on_its_lane_stream"] is True
    assert lanes["last_gather_steps"] == [9]
    for k, log in enumerate(lanes["lane_stream_logs"]):
        steps = [e[1] for e in log if isinstance(e, list)]
        assert steps == list(range(k + 1, 10, 3)), (k, log)
        assert log == [x for s in steps for x in ("event", ["forward", s], "event")], (k, log)
    assert j["gather_check"] == {"gathered_rows": 6, "every_rank_slice_equals_local": True}
