"""Run the exhaustive fast-reciprocal self-test on cuda:0 (see include/acmmp.h)."""
import ctypes as C, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from acmmp_amd import _abi
lib = _abi.load_library()
m, n = C.c_uint64(), C.c_uint64()
t0 = time.perf_counter()
rc = lib.acmmp_selftest_reciprocal(0, C.byref(m), C.byref(n))
print(json.dumps({"rc": rc, "mismatches": m.value, "checked": n.value, "seconds": time.perf_counter() - t0}))
