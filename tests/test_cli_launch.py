"""Launch hygiene of the multi-process CLI: the forkserver that
spawns one process per GPU must start before the CLI makes any HIP call (gpu_count,
engines), so no rank is ever fork+exec'ed from a GPU-initialised process
(ref launch: pfsp_dist_multigpu_cuda.c:907-919, one MPI rank per GPU)."""
import pytest

from dist_gpu_accelerated_tree_search_amd import cli, ops
from dist_gpu_accelerated_tree_search_amd.parallel import launch


@pytest.mark.parametrize("argv,want", [
    (["pfsp", "-D", "2", "-C", "0"], True),
    (["pfsp", "-D", "2"], False),                      # -C 1: one process drives every GPU
    (["pfsp", "-D", "4", "-C", "0", "--single-process"], False),
    (["pfsp", "-D", "2", "-C", "0", "--gpus-list", "0,1"], False),
    (["pfsp", "-D", "1", "-C", "0"], False),
    (["pfsp", "--D=3", "--C=0"], True),
    (["nqueens", "-N", "12", "-D", "2"], True),
    (["nqueens", "-N", "12"], False),
    (["pfsp", "-D2", "-C0"], True),                    # joined short options
    (["pfsp", "-D", "2", "-C", "2"], True),            # same routing test as pfsp_main (C != 1)
    (["pfsp", "-D", "3", "-C", "0", "--single"], False),  # abbreviated --single-process
    (["pfsp", "-D", "0", "-C", "4"], False),           # CPU only
    (["nqueens", "-D3"], True),
])
def test_spawn_planned(argv, want, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert cli._spawn_planned(argv) is want


def test_spawn_planned_under_torchrun(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert cli._spawn_planned(["pfsp", "-D", "2", "-C", "0"]) is False


def test_forkserver_starts_before_any_gpu_call(monkeypatch, capsys):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    calls = []
    monkeypatch.setattr(launch, "warm_forkserver", lambda: calls.append("forkserver"))

    def fake_count():
        calls.append("gpu_count")
        return 0  # no device: the CLI stops with the reference's message

    monkeypatch.setattr(ops, "gpu_count", fake_count)
    rc = cli.main(["pfsp", "-i", "14", "-D", "2", "-C", "0", "--no-csv"])
    assert rc == 1
    assert "More GPU devices requested" in capsys.readouterr().out
    assert calls[0] == "forkserver" and calls[-1] == "gpu_count" and calls.count("gpu_count") == 1, calls


def test_spawn_local_refuses_forkserver_after_hip(monkeypatch):
    monkeypatch.setattr(launch, "_WARM", False)
    monkeypatch.setattr(launch, "hip_touched", lambda: True)
    with pytest.raises(RuntimeError, match="forkserver"):
        launch.spawn_local(2, print)


def test_device_needs_gloo(capsys):
    with pytest.raises(SystemExit):
        cli.main(["pfsp", "-D", "2", "-C", "0", "--device", "0", "--no-csv"])
    assert "--comm gloo" in capsys.readouterr().err


def test_rank_spec_device_needs_gloo():
    from dist_gpu_accelerated_tree_search_amd.parallel.workers import solve_rank

    with pytest.raises(ValueError, match="gloo"):
        solve_rank({"problem": "pfsp", "backend": "gpu", "device": 0, "comm": "nccl"})


def test_heuristic_ub_is_opt_in_and_recorded(tmp_path, monkeypatch, capsys):
    # -u 0 prints "inf" (the reference's semantics) unless --heuristic-ub asks for the host
    # heuristics' incumbent, which is then printed and recorded (CPU run: -D 0 ignores it)
    import json

    from dist_gpu_accelerated_tree_search_amd.models.pfsp import PfspModel
    from dist_gpu_accelerated_tree_search_amd.utils import report

    monkeypatch.delenv("TTS_DIVE", raising=False)
    assert "Initial upper bound: inf" in report.pfsp_settings(14, 10, 20, 0, 1, 1, 0, 1, 1, 1, 2, None)
    assert "heuristic (1400)" in report.pfsp_settings(14, 10, 20, 0, 1, 1, 0, 1, 1, 1, 2, 1400)

    class A:
        ub, D, heuristic_ub = 0, 1, False

    m = PfspModel(14, 1)
    assert cli._init_ub(A, m) is None
    A.heuristic_ub = True
    monkeypatch.setenv("TTS_DIVE", "32")
    assert 1377 <= cli._init_ub(A, m) < 1500
    A.ub = 1
    assert cli._init_ub(A, m) == 1377
    out = tmp_path / "r.json"
    monkeypatch.delenv("TTS_DIVE", raising=False)
    assert cli.main(["pfsp", "-i", "2", "-l", "1", "-u", "0", "-D", "0", "--no-csv", "--json", str(out)]) == 0
    assert "Initial upper bound: inf" in capsys.readouterr().out
    rec = json.loads(out.read_text().splitlines()[-1])
    assert rec["initial_ub"] is None and rec["best"] == 1359


def test_console_entry_point_resolves():
    # pyproject's `tts` script is the CLI's main (pip install -e . puts it on PATH)
    import importlib
    import os

    import tomli

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "pyproject.toml"), "rb") as f:
        meta = tomli.load(f)
    mod, fn = meta["project"]["scripts"]["tts"].split(":")
    assert getattr(importlib.import_module(mod), fn) is cli.main
