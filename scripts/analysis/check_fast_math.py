"""Every float bit pattern through ldsp_debug_math_fastcheck (host build of
ldsp_math.hpp): lm_logf_fast / lm_expf_fast must equal lm_logf / lm_expf bit for
bit on their whole fast ranges.  ~1 minute on 8 threads."""
import ctypes as C
import os
import sys
from concurrent.futures import ThreadPoolExecutor

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "python-liquiddsp_amd", "libldsp.so"))
parts = 64
step = (1 << 32) // parts


def run(fn, p):
    c, b = C.c_uint64(), C.c_uint64()
    end = min((p + 1) * step, 0xFFFFFFFF)
    assert lib.ldsp_debug_math_fastcheck(fn, p * step, end, 1, C.byref(c), C.byref(b)) == 0
    return c.value, b.value


with ThreadPoolExecutor(os.cpu_count() or 8) as ex:
    for fn, name in ((0, "logf"), (1, "expf")):
        res = list(ex.map(lambda p: run(fn, p), range(parts)))
        print(name, "checked", sum(r[0] for r in res), "mismatches", sum(r[1] for r in res), flush=True)
        if any(r[1] for r in res):
            sys.exit(1)
