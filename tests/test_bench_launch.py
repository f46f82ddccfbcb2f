"""bench.py --gpus N without an outer launcher: it starts its N ranks itself (torch.distributed.run as
a child process) and relays rank 0's JSON line.  Exercised on CPU with FEDML_AMD_BENCH_CPU_PROBE=1,
where each rank only joins a gloo group and sums its rank (no GPU is touched)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, extra_env=None, timeout=240):
    env = dict(os.environ, FEDML_AMD_BENCH_CPU_PROBE="1")
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_relays_rank0_line(n):
    r = _run(["--gpus", str(n), "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == n
    assert lines[0]["rank_sum"] == sum(range(n))


def test_self_launch_propagates_rank_failure():
    r = _run(["--gpus", "2"], {"FEDML_AMD_BENCH_CPU_PROBE_FAIL_RANK": "1"})
    assert r.returncode != 0  # rank 0 may have printed its line already; the run still fails


def test_stage_watchdog_ends_a_hung_rank():
    r = _run(["--gpus", "2", "--stage-timeout", "3"], {"FEDML_AMD_BENCH_CPU_PROBE_HANG_RANK": "1"})
    assert r.returncode != 0
    assert "no progress" in r.stderr and "probe hang" in r.stderr


def test_launch_timeout_kills_the_group():
    r = _run(["--gpus", "2", "--stage-timeout", "0", "--launch-timeout", "8"],
             {"FEDML_AMD_BENCH_CPU_PROBE_HANG_RANK": "0"})
    assert r.returncode == 124
    assert "exceeded" in r.stderr


def test_launch_cmd_shape():
    import bench
    cmd = bench.launch_cmd(4, ["--gpus", "4", "--steps", "5"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["--gpus", "4", "--steps", "5"][-3:]
    assert cmd[cmd.index("--master-port") + 1] == "29555"


def test_roofline_block_multi_gpu_is_whole_step():
    import bench
    wl = {"name": "fedavg_flat_K128_P125000000_fp32_tiled"}
    b = bench.roofline_block(wl, 8, 40000.0, "GB/s", 6000.0, 1.3, 8.2e9)
    assert b["peak"] == 8 * bench.HBM_PEAK_GBS
    assert b["frac"] == round(40000.0 / (8 * bench.HBM_PEAK_GBS), 4)
    assert b["local_kernel"]["frac"] == round(6000.0 / bench.HBM_PEAK_GBS, 4)
    one = bench.roofline_block(wl, 1, 6600.0, "GB/s", 6650.0, 9.7, 64.5e9)
    assert one["frac"] == round(6650.0 / bench.HBM_PEAK_GBS, 4) and "local_kernel" not in one
    if one["traffic"] is not None:
        assert "not measured in this run" in one["traffic_source"]


def test_self_launch_at_one_rank():
    """--self-launch forces the launcher chain at --gpus 1 (what the driver's scaling run executes)."""
    r = _run(["--gpus", "1", "--self-launch", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 1


def test_prelaunch_device_count_never_touches_hip(monkeypatch):
    """The parent counts GPUs from sysfs / device nodes: with every HIP-backed count made to raise,
    main() still reaches the launcher (stubbed) -- nothing initialises HIP before the ranks start."""
    import torch
    import bench

    def boom(*a, **k):
        raise AssertionError("HIP device count called in the launcher parent")
    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom, raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", boom)
    monkeypatch.setattr(torch.cuda, "init", boom)
    assert bench.visible_gpu_count() is None or isinstance(bench.visible_gpu_count(), int)
    calls = []
    monkeypatch.setattr(bench, "visible_gpu_count", lambda: 8)
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv, t, script=None: calls.append((n, list(argv))) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_CPU_PROBE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_REHEARSAL", raising=False)
    for argv in (["--gpus", "8"], ["--gpus", "1", "--self-launch", "--loopback"]):
        monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
        with pytest.raises(SystemExit) as e:
            bench.main()
        assert e.value.code == 0
    assert calls == [(8, ["--gpus", "8"]), (1, ["--gpus", "1", "--self-launch", "--loopback"])]


def test_prelaunch_refuses_more_ranks_than_gpus(monkeypatch):
    import bench
    monkeypatch.setattr(bench, "visible_gpu_count", lambda: 1)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_CPU_PROBE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_REHEARSAL", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "only 1" in str(e.value.code)


def test_visible_gpu_count_honours_visible_devices(monkeypatch, tmp_path):
    import glob as _glob
    import bench
    # a fake KFD topology: a CPU node, two GPU nodes (render nodes absent here: counted)
    root = tmp_path / "nodes"
    for i, simd in enumerate([0, 1024, 1024]):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"simd_count {simd}\ndrm_render_minor {128 + i}\n")
    real = _glob.glob
    monkeypatch.setattr(_glob, "glob", lambda pat: real(str(root / "*" / "properties"))
                        if pat.startswith("/sys/class/kfd") else [])
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    assert bench.visible_gpu_count() == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.visible_gpu_count() == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")  # explicitly empty: no device
    assert bench.visible_gpu_count() == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setattr(_glob, "glob", lambda pat: [])  # nothing readable: unknown
    assert bench.visible_gpu_count() is None
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", " , ")
    assert bench.visible_gpu_count() == 0


def test_prelaunch_refuses_with_empty_visible_mask(monkeypatch):
    """An explicitly empty *_VISIBLE_DEVICES is 0 devices, not "unknown": the launcher refuses early."""
    import bench
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_CPU_PROBE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_REHEARSAL", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", lambda *a, **k: pytest.fail("launched with no visible GPU"))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "only 0" in str(e.value.code)


def test_unknown_gpu_count_does_not_refuse(monkeypatch):
    """None = the parent could not tell (no readable topology): it launches and lets the ranks report."""
    import bench
    monkeypatch.setattr(bench, "visible_gpu_count", lambda: None)
    calls = []
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv, t, script=None: calls.append(n) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_CPU_PROBE", raising=False)
    monkeypatch.delenv("FEDML_AMD_BENCH_REHEARSAL", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and calls == [8]
