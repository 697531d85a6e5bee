"""The loopback transport (gqmap_debug_loop_*, not in the public header): n
column-strip tile contexts in one process, one host thread each, whose RCCL
iteration code runs with real neighbours on one GPU -- only the three NCCL
calls (grouped ncclSend/ncclRecv, the two ncclAllGather) are replaced by
device copies between the ranks' buffers (gqmap_engine.hip LoopGroup)."""
import ctypes as C
import threading


def _lib():
    from gqmap_opticalflow_amd import _lib as L
    lib = L.load()
    lib.gqmap_debug_loop_create.restype = C.c_void_p
    lib.gqmap_debug_loop_create.argtypes = [C.c_int, C.c_int]
    lib.gqmap_debug_loop_destroy.restype = None
    lib.gqmap_debug_loop_destroy.argtypes = [C.c_void_p]
    lib.gqmap_debug_loop_calls.restype = C.c_ulonglong
    lib.gqmap_debug_loop_calls.argtypes = [C.c_void_p]
    lib.gqmap_debug_tile_attach_loop.restype = C.c_int
    lib.gqmap_debug_tile_attach_loop.argtypes = [C.c_void_p, C.c_void_p]
    return lib


class LoopGroup:
    """A loopback communicator of n ranks on `device`; attach(tile_engine)
    for every tile 0..n-1, then drive each rank from its own thread
    (ranks())."""

    def __init__(self, n, device=0):
        self.lib = _lib()
        self.n = n
        self.h = self.lib.gqmap_debug_loop_create(n, device)
        if not self.h:
            raise RuntimeError("gqmap_debug_loop_create failed")

    def attach(self, eng):
        from gqmap_opticalflow_amd._lib import check
        check(self.lib.gqmap_debug_tile_attach_loop(eng.ctx, C.c_void_p(self.h)), "gqmap_debug_tile_attach_loop")

    def calls(self):
        return int(self.lib.gqmap_debug_loop_calls(C.c_void_p(self.h)))

    def destroy(self):
        if self.h:
            self.lib.gqmap_debug_loop_destroy(C.c_void_p(self.h))
            self.h = None


def ranks(fn, tiles, timeout=300):
    """fn(tile) on one thread per tile (the library calls release the GIL);
    returns the results in tile order, re-raising the first failure."""
    out = [None] * len(tiles)
    err = [None] * len(tiles)

    def body(i):
        try:
            out[i] = fn(tiles[i])
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            err[i] = e

    th = [threading.Thread(target=body, args=(i,), daemon=True) for i in range(len(tiles))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
        if t.is_alive():
            raise TimeoutError("a rank thread did not finish")
    for e in err:
        if e is not None:
            raise e
    return out
