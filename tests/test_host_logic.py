"""Host-side logic that needs no GPU: synthetic workloads, the roofline flop model, the
ABI parameter builders."""
import numpy as np

from cwbl import abi, synth


def test_flop_model_matches_survey():
    # F(40,200) = 1 230 400 flop
    assert synth.flops_per_point(40, 200) == 1_230_400
    assert synth.flops_total(40, 3, 600) == 3 * synth.flops_per_point(40, 200)


def test_synthetic_c2_shapes_and_determinism():
    a = synth.make("c2", scale=0.05, nz=4)
    b = synth.make("c2", scale=0.05, nz=4)
    assert a.var.shape == (40, 4, a.ny, a.nx) and a.var.dtype == np.float32
    assert a.alt.shape == (4, a.ny, a.nx)
    assert a.obs_xyz.shape == (a.obs.shape[0], 3) and a.hdxb.shape == (40, a.obs.shape[0])
    np.testing.assert_array_equal(a.var, b.var)
    np.testing.assert_array_equal(a.hdxb, b.hdxb)


def test_shards_are_the_reference_column_grid_of_the_full_grid():
    # letkf_local_info (module_mpi_util.f90:71-188): rank r = ix + iy*px of a px x py grid
    # (px >= py, MPI_Dims_create) owns columns x = ix + i*px, rows y = iy + j*py
    full = synth.make("c2", scale=0.05, nz=3)  # 15 x 15
    for world, (px, py) in ((1, (1, 1)), (3, (3, 1)), (4, (2, 2)), (6, (3, 2)), (8, (4, 2))):
        seen = np.zeros((full.ny, full.nx), np.int32)
        for r in range(world):
            part = synth.make("c2", scale=0.05, nz=3, shard=(r, world))
            ix, iy = r % px, r // px
            np.testing.assert_array_equal(part.var, full.var[:, :, iy::py, ix::px])
            np.testing.assert_array_equal(part.x, full.x[iy::py, ix::px])
            np.testing.assert_array_equal(part.alt, full.alt[:, iy::py, ix::px])
            np.testing.assert_array_equal(part.obs, full.obs)
            seen[iy::py, ix::px] += 1
        assert (seen == 1).all()
    # 300 x 300 (configs[1..2]) splits evenly over 1, 2, 4 and 8 ranks
    from cwbl.dist import shard_columns
    for world in (1, 2, 4, 8):
        sizes = {len(a) * len(b) for a, b in (shard_columns(300, 300, r, world)
                                               for r in range(world))}
        assert sizes == {90000 // world}


def test_var_params_defaults_follow_module_config():
    vp = abi.var_params(multi_infl=1.6, use_rtpp=1, rtpp_alpha=0.95)
    assert abs(vp.multi_infl - 1.6) < 1e-7 and vp.use_rtpp == 1 and vp.use_rtps == 0
    assert vp.gts[1].use_it == 0 and vp.radar[1].use_it == 0
    tp = abi.type_params(use_it=1, max_lz_pts=300, hclr=12.0, vclr=3.0, err_muti=[0.5] * 5,
                         is_assim=[1, 0, 1])
    assert list(tp.is_assim) == [1, 0, 1, 1, 1]
    assert tp.max_lz_pts == 300


def test_make_slab_rejects_arrays_the_abi_would_misread():
    # the library reads raw pointers and updates var in place: wrong dtype, strides or
    # memory kind must fail before the call
    import pytest
    nz, ny, nx, k = 2, 3, 4, 5
    x = np.zeros((ny, nx), np.float32)
    alt = np.zeros((nz, ny, nx), np.float32)
    var = np.zeros((k, nz, ny, nx), np.float32)
    abi.make_slab(x, x, alt, var)  # fine
    with pytest.raises(TypeError):
        abi.make_slab(x, x, alt, var.astype(np.float64))
    with pytest.raises(ValueError):
        abi.make_slab(x, x, alt, np.zeros((k, nz, nx, ny), np.float32).transpose(0, 1, 3, 2))
    with pytest.raises(TypeError):
        abi.make_slab(x, x, alt, var, memory=abi.MEM_DEVICE)  # host arrays as device pointers
    b = abi.ObsSetBuilder(abi.MEM_DEVICE)
    with pytest.raises(TypeError):
        b.add_radar(abi.RADAR_VR, np.zeros((2, 3), np.float32), np.zeros(2, np.float32),
                    np.zeros((k, 2), np.float32))
    # host mode converts (copies) instead
    abi.ObsSetBuilder().add_gts(abi.GTS_SYNOP, np.zeros((2, 3)), np.zeros((2, 5)),
                                np.ones((2, 5)), np.zeros((k, 2, 5)),
                                np.zeros((k, 2, 5), np.int64)).build()


def test_local_noise_shards_keep_the_geometry():
    full = synth.make("c2", scale=0.05, nz=3)
    for world in (2, 4):
        from cwbl.dist import shard_columns
        for r in range(world):
            part = synth.make("c2", scale=0.05, nz=3, shard=(r, world), local_noise=True)
            xs, ys = shard_columns(full.nx, full.ny, r, world)
            np.testing.assert_array_equal(part.x, full.x[np.ix_(ys, xs)])
            np.testing.assert_array_equal(part.alt, full.alt[:, ys][:, :, xs])
            np.testing.assert_array_equal(part.obs_xyz, full.obs_xyz)
            assert part.var.shape == (40, 3, len(ys), len(xs))


def test_bench_refuses_a_rank_count_that_is_not_gpus():
    """bench.py --gpus N must time N ranks: under a launcher whose WORLD_SIZE differs it
    exits non-zero before touching the GPU (--gpus was ignored)."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_roofline_block_takes_the_dominant_kernel_and_its_algorithmic_flops():
    """bench.py's roofline: the kernel with the largest summed HIP-event time, its part of
    letkf_solve's algorithmic flops (syrk + Yb d for the assembly; the dsytd2 steps' 4 n^2
    and 6k^2 for the reflector solve) over that time; F stays reference-equivalent detail."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    k, solved, nobs = 40, 1000, 216_000
    # the steps of dsytd2 sum to ~4k^3/3
    tri = bench._tri_flops(k, 0, k)
    assert tri == sum(4 * n * n for n in range(1, k)) and abs(tri / (4 * k ** 3 / 3) - 1) < 0.05
    kt = {"assemble_record_kernel<4>": {"launches": 2, "points": solved, "ms": 3.0},
          "solve_tq40_kernel<40, 0>": {"launches": 2, "points": solved, "ms": 2.0},
          "search_binned_kernel": {"launches": 2, "points": solved, "ms": 9.0}}
    roof, per = bench.roofline_block(kt, k, solved, nobs, 5.0, "no-such-config")
    assert roof["kernel"] == "assemble_record_kernel<4>"  # the search has no FP64 model
    want = nobs * (k * (k + 1) + 2 * k) / 3e-3 / 1e12
    assert abs(roof["achieved"] - want) < 1e-9 and roof["frac"] == roof["achieved"] / 78.6
    assert roof["avg_launch_ms"] == 1.5 and "algorithmic_tflops" not in per["search_binned_kernel"]
    tq = per["solve_tq40_kernel<40, 0>"]["algorithmic_tflops"]
    assert abs(tq - solved * (tri + 6 * k * k) / 2e-3 / 1e12) < 1e-9
    # the split k = 128 pair: steps 0..63 in the hand-off kernel, the rest in the tail
    a = bench.kernel_algorithmic_flops("solve_tq_big_kernel<128, false, 64>", 128, 1, 200)
    b = bench.kernel_algorithmic_flops("solve_tqb_tail_kernel<128, 64, 3>", 128, 1, 200)
    assert a + b == 200 * (128 * 129 + 256) + bench._tri_flops(128, 0, 128) + 6 * 128 * 128
    assert bench.kernel_algorithmic_flops("solve_tq_rows_kernel<128, 64>", 128, 1, 200) == a


def test_hbm_block_sums_pmc_bytes_per_step(monkeypatch):
    """roofline.hbm: PMC HBM bytes of every kernel x its calls / the profiled steps, over the
    live ms_per_step and 8 TB/s; the unique-bytes figure is 4 (2k + 3) B per point."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    pmc = {"_meta": {"steps": 2},
           "assemble_record_kernel<4>": {"hbm_bytes_per_launch": 3e9, "calls": 4},
           "solve_tq40_kernel<40, 0>": {"hbm_bytes_per_launch": 1e9, "calls": 4},
           "notes": "not a kernel"}
    monkeypatch.setattr(bench, "load_pmc", lambda config: (pmc, "t"))
    h = bench.hbm_block("c2", 40, 1_000_000, 10.0)
    assert h["pmc_bytes_per_step"] == (3e9 * 4 + 1e9 * 4) / 2
    assert abs(h["achieved_gbs"] - 8e9 / 1e-2 / 1e9) < 1e-9
    assert h["frac"] == h["achieved_gbs"] / bench.HBM_PEAK_GBS and bench.HBM_PEAK_GBS == 8000.0
    assert h["unique_bytes_per_step"] == 4.0 * 83 * 1_000_000
    assert h["by_kernel_bytes_per_step"]["assemble_record_kernel<4>"] == 6e9
    assert set(h["by_kernel_bytes_per_step"]) == {"assemble_record_kernel<4>",
                                                   "solve_tq40_kernel<40, 0>"}
    monkeypatch.setattr(bench, "load_pmc", lambda config: ({}, None))
    assert bench.hbm_block("no-such-config", 40, 1, 10.0) is None
    # the committed profile carries C2's figures
    monkeypatch.undo()
    assert bench.hbm_block("c2", 40, 1_000_000, 10.0)["pmc_bytes_per_step"] > 0


def test_baseline_process_count_follows_affinity_and_quota():
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n_aff, n_phys, quota = bench.host_cores()
    assert 1 <= n_phys <= n_aff == len(os.sched_getaffinity(0))
    procs, note = bench.baseline_procs()
    assert procs == (n_phys if quota is None else max(1, min(n_phys, int(quota))))
    assert f"{procs} used" in note


def _bench_json(stdout):
    import json
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert lines, stdout
    return json.loads(lines[-1])


def test_bench_failure_still_prints_a_json_line():
    """A run that fails (here by CWBL_BENCH_FAIL_AT's injection at the first stage; on a
    first RCCL run it would be process-group init or the obs broadcast) still ends in one
    parseable JSON line with value null, the exception and the stage it came from."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CWBL_BENCH_FAIL_AT="device")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 1, r.stderr[-2000:]
    d = _bench_json(r.stdout)
    assert d["value"] is None and d["stage"] == "device" and "injected" in d["error"]
    assert d["metric"].startswith("analysis grid-points/sec")


def test_bench_two_rank_failure_reports_from_rank_0():
    """The same under torch.distributed.run with two ranks (gloo, CPU): rank 0 prints the
    error line, the run exits non-zero, and nothing hangs."""
    import os
    import socket
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CWBL_BENCH_FAIL_AT="device", CWBL_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1",
                        f"--master-port={port}", os.path.join(repo, "bench.py"), "--gpus", "2",
                        "--steps", "1"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    d = _bench_json(r.stdout)
    assert d["value"] is None and d["stage"] == "device" and d["rank"] == 0
    assert d["config"]["ranks"] == 2
