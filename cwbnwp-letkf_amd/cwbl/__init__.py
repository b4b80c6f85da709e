"""cwbl — host-side Python binding of the MI355X LETKF analysis core (C ABI in
include/cwb_letkf_core.h).  The compute lives in the HIP library lib/libcwbl.so; this
package only marshals arrays (ctypes) and provides synthetic workloads for bench/tests."""
from .abi import (ABI_VERSION, Core, CwblError, ObsSetBuilder, make_slab, type_params,  # noqa: F401
                  var_params, load_library, MEM_HOST, MEM_DEVICE, Q1_REPLICATE, Q1_PER_TYPE)
