"""GPU: the host path's copy machinery alone, on the real runtime
(fory_rowfmt_internal_host_copies). These are the staged scenarios tests/c/host_copy_mock.cpp
runs against the late-DMA mock on the CPU: random pieces in both directions between pageable
host buffers and device buffers, on the context's three streams, from a byte to several
staging blocks. After each call every piece's bytes match, and a call that returns before its
drain (as an error return does) still leaves correct bytes.

The declared-buffer (call-scoped registration) variants run on the CPU mock only. In the
in-process GPU suite they added ~50 register / unregister cycles of 24 MiB numpy buffers,
interleaved with torch's pageable copies, and the next test file's first tree-engine
case then hit an illegal address (profiles/r06/intermittent/README.md §4). Call-scoped
registration on the GPU is covered by tests/test_gpu_host.py's registration cases."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from fury_amd import workloads as W  # noqa: E402
from fury_amd.format.native import HostPipeline, NativePlan  # noqa: E402

pytestmark = pytest.mark.gpu


def _internal(name, restype, argtypes):
    from fury_amd import _lib
    f = getattr(_lib.load(), name)
    f.restype, f.argtypes = restype, argtypes
    return f


def _copies():
    P = ctypes.c_void_p
    return _internal("fory_rowfmt_internal_host_copies", ctypes.c_int,
                     [P, ctypes.c_int32, P, P, P, P, P, ctypes.c_int32, P, P, ctypes.c_int32])


def _call_regs(hp):
    f = _internal("fory_rowfmt_internal_host_call_regs", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p])
    out = np.zeros(3, np.int64)
    return f(hp.handle, out.ctypes.data)


@pytest.mark.parametrize("declare,flags", [(False, 0), (False, 1)])
@pytest.mark.parametrize("seed", [1, 2])
def test_host_copies_random_pieces(seed, declare, flags):
    rng = np.random.default_rng(seed)
    hp = HostPipeline(NativePlan(W.mixed_schema()), chunk_rows=1 << 16)
    copies = _copies()
    try:
        for call in range(3):
            nbuf, size = 3, (24 << 20) + int(rng.integers(0, 4096))
            host = [np.empty(size + 64, np.uint8)[int(rng.integers(0, 64)):][:size] for _ in range(nbuf)]  # unaligned starts
            dev = [torch.empty(size, dtype=torch.uint8, device="cuda") for _ in range(nbuf)]
            for h, d in zip(host, dev):  # distinct random contents on both sides
                h[:] = rng.integers(0, 256, size, dtype=np.uint8)
                d.copy_(torch.from_numpy(rng.integers(0, 256, size, dtype=np.uint8)))
            torch.cuda.synchronize()
            dsts, srcs, ns, kinds, streams, want = [], [], [], [], [], []
            cursor = [0] * nbuf
            for _ in range(120):
                w = int(rng.integers(0, nbuf))
                n = int(rng.integers(1, 64)) if rng.random() < 0.3 else int(rng.integers(1, 3 << 20))
                n = min(n, size - cursor[w])
                if n <= 0:
                    continue
                a = cursor[w]
                kind = int(rng.integers(1, 3))
                hp_ptr = host[w].ctypes.data + a
                dp_ptr = dev[w].data_ptr() + a
                if kind == 1:
                    dsts.append(dp_ptr), srcs.append(hp_ptr), want.append(("dev", w, a, host[w][a:a + n].copy()))
                else:
                    dsts.append(hp_ptr), srcs.append(dp_ptr), want.append(("host", w, a, None))
                ns.append(n), kinds.append(kind), streams.append(int(rng.integers(0, 3)))
                cursor[w] += n + (int(rng.integers(0, 512)) if rng.random() < 0.3 else 0)
            dev_before = [d.cpu().numpy() for d in dev]
            for i, (side, w, a, _) in enumerate(want):
                if side == "host":
                    want[i] = ("host", w, a, dev_before[w][a:a + ns[i]].copy())
            k = len(ns)
            arr = lambda xs, t: (t * k)(*xs)  # noqa: E731
            decl = (ctypes.c_void_p * nbuf)(*[h.ctypes.data for h in host]) if declare else None
            decl_n = (ctypes.c_int64 * nbuf)(*[size] * nbuf) if declare else None
            rc = copies(hp.handle, k, arr(dsts, ctypes.c_void_p), arr(srcs, ctypes.c_void_p), arr(ns, ctypes.c_int64),
                        arr(kinds, ctypes.c_int32), arr(streams, ctypes.c_int32), nbuf if declare else 0, decl, decl_n,
                        flags)
            assert rc == 0
            dev_after = [d.cpu().numpy() for d in dev]
            for i, (side, w, a, exp) in enumerate(want):
                got = dev_after[w][a:a + ns[i]] if side == "dev" else host[w][a:a + ns[i]]
                assert np.array_equal(got, exp), (call, i, side, ns[i], streams[i])
            assert _call_regs(hp) == 0
    finally:
        hp.close()
