"""DbSink.consume_encoded on a rollover-sized blob of COPY rows (40 MB): wall time per call."""
import random
import sys
import time

sys.path.insert(0, ".")
from apmbackend_amd import _native  # noqa: E402

N = _native.load(build_if_missing=False)
rng = random.Random(1)
rows = [("2020-01-07 10:00:00.000+00\tjvm00\tgetSvc%05d\t12.5\t360\t{\"average\":%d,\"averageavg\":1.5}" % (i % 10000, i))
        + "x" * rng.randint(100, 200) + "\n" for i in range(160000)]
blob = "".join(rows).encode()
s = N.DbSink(1000, 1e9, ["t_tx", "t_fs", "t_al", "t_jx", "t_fb"], ["a", "b", "c", "d", "e"], "null", [], 1 << 62, 8)
for rep in range(5):
    t = time.perf_counter()
    s.consume_encoded(1, blob)
    t1 = time.perf_counter()
    s.drain()
    print("consume ms", round((t1 - t) * 1e3, 2), flush=True)
p = N.alloc_pinned(len(blob) + 64)
N.memcpy_to(p, blob, 0)
for rep in range(5):
    t = time.perf_counter()
    s.consume_encoded_ptr(1, p, len(blob))
    t1 = time.perf_counter()
    s.drain()
    print("pinned consume ms", round((t1 - t) * 1e3, 2), flush=True)
N.free_pinned(p)
