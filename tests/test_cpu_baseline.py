"""bench.py's CPU baselines on a small block of the synthetic grid (CPU only).

The reference CPU baseline runs the reference's own compiled code (oracle/_ref/ref_harness,
driver mode) on blocks of whole columns; its input is written by bench._ref_driver_blob.  The
harness output must equal the C restatement (oracle/liboracle.so) on the same block bit for
bit, which pins the blob layout (the harness only exists where /root/reference was built).
"""
import ctypes as C
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from cwbl import abi, synth
from helpers import REPO, oracle

sys.path.insert(0, REPO)
import bench  # noqa: E402


def _oracle_block(w, i0, j0, nb):
    sub = lambda a: np.ascontiguousarray(a[..., j0:j0 + nb, i0:i0 + nb])  # noqa: E731
    var = sub(w.var).copy()
    slab = abi.make_slab(sub(w.x), sub(w.y), sub(w.alt), var)
    ob = abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build()
    st = abi.Stats()
    rc = oracle().orc_analyze_var(w.k, 0, -5.0, 0, C.byref(ob), C.byref(w.vp), C.byref(slab), 1,
                                  C.byref(st))
    assert rc == 0
    return var, st


@pytest.mark.skipif(not os.path.exists(bench.REF_HARNESS), reason="reference harness not built")
def test_reference_harness_block_equals_oracle():
    w = synth.make("c2", scale=0.06, nz=4)
    nb, i0, j0 = 5, 3, 4
    with tempfile.TemporaryDirectory() as td:
        with open(os.path.join(td, "in.bin"), "wb") as f:
            f.write(bench._ref_driver_blob(w, i0, j0, nb))
        env = dict(os.environ, MKL_CBWR="COMPATIBLE", MKL_THREADING_LAYER="SEQUENTIAL",
                   MKL_NUM_THREADS="1")
        subprocess.run([bench.REF_HARNESS, "driver", "in.bin", "out.bin"], cwd=td, env=env,
                       check=True, stdout=subprocess.DEVNULL)
        got = np.fromfile(os.path.join(td, "out.bin"), np.float32)
    want, st = _oracle_block(w, i0, j0, nb)
    assert st.solved > 0
    # out.bin is var(nx, ny, nz, 0:k-1) in Fortran order == the C-order (k, nz, ny, nx) slab
    np.testing.assert_array_equal(got.view(np.uint32), want.ravel().view(np.uint32))


def test_port_baseline_runs_on_a_small_grid():
    w = synth.make("c2", scale=0.04, nz=3)
    out = bench.cpu_baseline(w, target_s=0.05)
    assert out["kind"] == "port" and out["value"] > 0 and out["cores"] >= 1
