#!/usr/bin/env python3
"""Bitwise comparison of two library builds on one C2-shaped case (a kernel change that should
leave every result bit unchanged): python scripts/lib_bitcmp.py OUT.npy [nx] [config]  analyses one
variable with the library CWBL_LIBRARY names and saves the slab; --cmp A.npy B.npy compares."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "cwbnwp-letkf_amd"))

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    diff = int((a.view(np.uint32) != b.view(np.uint32)).sum())
    print(f"{sys.argv[2]} vs {sys.argv[3]}: {diff} of {a.size} words differ")
    sys.exit(1 if diff else 0)

from cwbl import abi, synth  # noqa: E402

nx = int(sys.argv[2]) if len(sys.argv) > 2 else 100
cfg = sys.argv[3] if len(sys.argv) > 3 else "c2"
w = synth.make(cfg, nx=nx, ny=nx)
c = abi.Core(w.k, device=0)
c.set_obs(abi.ObsSetBuilder().add_radar(w.radar_type, w.obs_xyz, w.obs, w.hdxb).build())
var = w.var.copy()
st = c.analyze_var(w.vp, abi.make_slab(w.x, w.y, w.alt, var))
c.finalize()
np.save(sys.argv[1], var)
print(f"{os.environ.get('CWBL_LIBRARY', 'in-tree')}: solved {st.solved}, nobs {st.nobs_sum}")
