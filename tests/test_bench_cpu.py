"""bench.py host logic that needs no GPU: how timed frames are grouped into
multi-frame launches (mm_trace_tile_frames), and which PMC record a bench line
may quote (the one of its own sources and launch shape)."""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


@pytest.mark.parametrize("count,per,expect", [
    (10, 8, [5, 5]), (16, 8, [8, 8]), (17, 8, [5, 6, 6]), (3, 8, [3]), (1, 8, [1]), (0, 8, []), (9, 1, [1] * 9),
])
def test_launch_sizes(count, per, expect):
    from bench import launch_sizes

    sizes = launch_sizes(count, per)
    assert sizes == expect
    assert sum(sizes) == count and all(0 < s <= per for s in sizes)
    assert max(sizes, default=0) - min(sizes, default=0) <= 1


def _args(config="c3", emulate_ranks=0):
    from types import SimpleNamespace

    return SimpleNamespace(config=config, emulate_ranks=emulate_ranks, pipeline="auto", opt=[])


def test_pmc_record_of_the_same_sources_is_used(monkeypatch):
    """profiles/pmc_<config>.json counts only for the sources it was taken on;
    its lane-ops and HBM bytes scale to the run's frames per launch."""
    import json

    import bench

    rec = json.loads((bench.REPO / "profiles" / "pmc_c3.json").read_text())
    monkeypatch.setattr(bench, "src_hash", lambda: rec["src_hash"])
    m, traffic = bench.pmc_profile(_args(), rec["frames_per_launch"] * 2, 0.1, 1)
    assert m["source"] == "profiles/pmc_c3.json" and not m.get("stale")
    assert traffic == round(rec["hbm_bytes_per_launch"] * 2)
    assert m["valu_lane_ops_tops"] == round(rec["valu_lane_ops_per_launch"] * 2 / 0.1 / 1e12, 3)


def test_pmc_record_of_other_sources_is_marked_stale(monkeypatch):
    import bench

    monkeypatch.setattr(bench, "src_hash", lambda: "0" * 16)
    m, traffic = bench.pmc_profile(_args(), 20, 0.05, 1)
    assert m["stale"] is True and traffic is None and "stale_valu_lane_ops_tops" in m


def test_pmc_record_per_emulated_rank_share(monkeypatch):
    """--emulate-ranks N and world = N both read pmc_<config>_r<N>.json (rank
    0's own launch shape), not the whole frame's record; without one there is
    no record."""
    import json

    import bench

    rec = json.loads((bench.REPO / "profiles" / "pmc_c3_r8.json").read_text())
    monkeypatch.setattr(bench, "src_hash", lambda: rec["src_hash"])
    m, _ = bench.pmc_profile(_args(emulate_ranks=8), 20, 0.0065, 1)
    assert m["source"] == "profiles/pmc_c3_r8.json"
    m, _ = bench.pmc_profile(_args(), 20, 0.0065, 8)  # world = 8: rank 0's launch shape, the same record
    assert m["source"] == "profiles/pmc_c3_r8.json"
    m, traffic = bench.pmc_profile(_args(), 20, 0.013, 3)  # no record of rank 0 of 3
    assert m["source"] is None and traffic is None
    m, _ = bench.pmc_profile(_args(), 20, 0.0065, 8, shared=True)  # diagnostics: never a roofline
    assert m["source"] is None


def _frac_keys(d, path=""):
    """Every (path, value) of a key named "frac" in a nested dict."""
    out = []
    for k, v in d.items():
        if isinstance(v, dict):
            out += _frac_keys(v, f"{path}.{k}")
        elif k == "frac" and v is not None:
            out.append((f"{path}.{k}", v))
    return out


def test_roofline_at_eight_ranks_is_the_executed_basis(monkeypatch):
    """the N = 8 line's roofline reads rank 0's PMC record
    (pmc_c3_r8.json) and quotes executed lane-ops like N = 1 -- at the
    record's own launch time its frac equals the record's profile_frac within
    1 % -- and no printed fraction passes 1 (the models carry model_ratio)."""
    import json

    import bench

    rec = json.loads((bench.REPO / "profiles" / "pmc_c3_r8.json").read_text())
    monkeypatch.setattr(bench, "src_hash", lambda: rec["src_hash"])
    k_avg = rec["kernel_avg_ms"] / 1e3
    fpl = rec["frames_per_launch"]
    m, traffic = bench.pmc_profile(_args(), fpl, k_avg, 8)
    # a reference-walk model far above the peak and an HBM model above it: printed as ratios only
    r = bench.roofline(120e12 * k_avg, 9e12 * k_avg, k_avg, 1, fpl, m, traffic, 1, {})
    assert r["basis"].startswith("executed") and "pmc_c3_r8.json" in r["basis"]
    assert abs(r["frac"] / m["profile_frac"] - 1) < 0.01, (r["frac"], m["profile_frac"])
    assert r["unit"] == "T lane-ops/s"
    assert r["reference_equivalent"]["model_ratio"] > 1 and r["model_hbm"]["model_ratio"] > 1
    fracs = _frac_keys(r)
    assert fracs and all(0 <= v <= 1 for _, v in fracs), fracs


def test_roofline_without_a_record_is_null_not_a_model():
    import bench

    m = {"source": None, "note": "no PMC record for this launch shape"}
    r = bench.roofline(40e12 * 0.05, 1e9, 0.05, 1, 20, m, None, 1, {})
    assert r["achieved"] is None and r["frac"] is None and r["basis"].startswith("none")
    assert r["reference_equivalent"]["model_ratio"] == round(40 / bench.VALU_PEAK_TOPS, 4)


def _largs(gpus=1, launcher="auto"):
    from types import SimpleNamespace

    return SimpleNamespace(gpus=gpus, launcher=launcher)


def test_gpus_n_without_a_launcher_starts_one_process_per_gpu():
    """`bench.py --gpus 8` run on its own must run 8 GPUs,
    not trace on one and print n_gpus 1.  Before torch or a GPU is touched it
    starts torch.distributed.run with one process per GPU as a child (never
    exec), with the same arguments; at N = 1 it runs in place unless
    --launcher torchrun asks for the multi-GPU path at one rank."""
    import bench

    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    how, cmd = bench.launch_plan(_largs(8), {}, argv, port=29577)
    assert how == "child"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29577"
    assert cmd[-len(argv) - 1:] == [str(bench.REPO / "bench.py")] + argv
    assert bench.launch_plan(_largs(1), {}, ["--gpus", "1"]) == ("run", None)
    how, cmd = bench.launch_plan(_largs(1, "torchrun"), {}, ["--gpus", "1", "--launcher", "torchrun"], port=1)
    assert how == "child" and "--nproc-per-node=1" in cmd


def test_gpus_must_match_the_launcher_world_size():
    """Under a launcher (WORLD_SIZE set -- the driver's torchrun) the child
    runs in place when WORLD_SIZE equals --gpus and refuses otherwise, so
    n_gpus always equals --gpus."""
    import bench

    assert bench.launch_plan(_largs(8), {"WORLD_SIZE": "8"}, []) == ("run", None)
    assert bench.launch_plan(_largs(1, "torchrun"), {"WORLD_SIZE": "1"}, []) == ("run", None)
    how, msg = bench.launch_plan(_largs(8), {"WORLD_SIZE": "2"}, [])
    assert how == "error" and "WORLD_SIZE=2" in msg and "--gpus 8" in msg
    how, _ = bench.launch_plan(_largs(0), {}, [])
    assert how == "error"


def test_mismatch_exits_nonzero_before_touching_a_gpu():
    """The refusal is an exit status, printed to stderr, with no JSON line."""
    import os
    import subprocess

    import bench

    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(bench.REPO / "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       env=env, timeout=120)
    assert p.returncode == 2 and p.stdout == "" and "WORLD_SIZE=4" in p.stderr


def test_child_relay_passes_rank0_line_and_exit_status(tmp_path):
    """relay_child: the child's JSON line is the one stdout line; other
    stdout goes to stderr; a failing child's status is the parent's."""
    import bench

    script = tmp_path / "c.py"
    script.write_text('import json,sys\nprint("banner")\nprint(json.dumps({"metric": "m", "value": 1}))\n'
                      'sys.exit(int(sys.argv[1]))\n')
    assert bench.relay_child([sys.executable, str(script), "0"]) == 0
    assert bench.relay_child([sys.executable, str(script), "3"]) == 3
    script.write_text("print('no line')\n")
    assert bench.relay_child([sys.executable, str(script)]) == 1


def test_stale_record_is_never_the_headline():
    """with a PMC record of other sources the roofline headline
    is null (never a model); the stale lane-ops rate sits
    only in the labelled stale_profile sub-object and the line carries
    stale: true."""
    import bench

    measured = {"source": "profiles/pmc_c3.json", "stale": True, "stale_valu_lane_ops_tops": 30.0}
    r = bench.roofline(40e12 * 0.05, 1e9, 0.05, 1, 20, measured, None, 1, {})
    assert r["stale"] is True and r["achieved"] is None and r["frac"] is None and r["basis"].startswith("none")
    assert r["stale_profile"]["valu_lane_ops_tops"] == 30.0
    fresh = bench.roofline(40e12 * 0.05, 1e9, 0.05, 1, 20, {"valu_lane_ops_tops": 29.0, "source": "x"}, 5, 1, {})
    assert fresh["stale"] is False and fresh["achieved"] == 29.0 and fresh["stale_profile"] is None
