"""Host-side costs of the HIP calls an engine's creation makes (GPU box): hipMalloc,
hipHostMalloc, hipStreamCreate, a pageable 2-D copy of 64 MT states, the same as one
contiguous copy, and zc_engine_create / destroy themselves."""
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

hip = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p


def t_us(fn, n=20):
    fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return 1e6 * (time.perf_counter() - t) / n


hip.hipSetDevice(0)
ptrs = []


def mall(b):
    p = vp()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(b)) == 0
    ptrs.append(p)


def free_all():
    for p in ptrs:
        hip.hipFree(p)
    ptrs.clear()


for b in (16, 4096, 1 << 20, 64 << 20):
    print(f"hipMalloc({b}) {t_us(lambda: mall(b)):.1f} us", flush=True)
    t = time.perf_counter()
    free_all()
    print(f"  hipFree x21 {1e6 * (time.perf_counter() - t) / 21:.1f} us each", flush=True)
hp = vp()
t = time.perf_counter()
hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(8192), 0)
t1 = time.perf_counter()
hip.hipHostFree(hp)
print(f"hipHostMalloc(8192) {1e6 * (t1 - t):.1f} us, hipHostFree {1e6 * (time.perf_counter() - t1):.1f} us", flush=True)
s = vp()
t = time.perf_counter()
hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
t1 = time.perf_counter()
hip.hipStreamDestroy(s)
print(f"hipStreamCreate {1e6 * (t1 - t):.1f} us, destroy {1e6 * (time.perf_counter() - t1):.1f} us", flush=True)
hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
d = vp()
hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(64 * 4096))
host = (ctypes.c_uint32 * (64 * 1024))()
sz = ctypes.c_size_t


def copy2d():
    hip.hipMemcpy2DAsync(d, sz(4096), host, sz(624 * 4), sz(624 * 4), sz(64), 1, s)
    hip.hipStreamSynchronize(s)


def copy1d():
    hip.hipMemcpyAsync(d, host, sz(64 * 4096), 1, s)
    hip.hipStreamSynchronize(s)


print(f"hipMemcpy2DAsync 64 x 624 words (pageable) {t_us(copy2d):.1f} us", flush=True)
print(f"hipMemcpyAsync 64 x 1024 words (pageable) {t_us(copy1d):.1f} us", flush=True)

from zeroclone_amd import _native  # noqa: E402

for g in (1, 64, 4096):
    for rep in range(3):
        t = time.perf_counter()
        ne = _native.NativeEngine(max_games=g, max_sims=100, max_batch=32, device=0)
        t1 = time.perf_counter()
        ne.close()
        print(f"NativeEngine({g} games) {1e3 * (t1 - t):.2f} ms, close {1e3 * (time.perf_counter() - t1):.2f} ms",
              flush=True)
