"""ctypes driver for the MEX gateways (mex/*.cpp) built against the MEX API
shim (tests/native/mexshim): builds MATLAB-style arguments, calls a
gateway's mexFunction, returns its outputs as numpy arrays.  Test
infrastructure only; MATLAB is not in this image."""
import ctypes as C
import os
import subprocess

import numpy as np

NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
_P = C.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", NATIVE, "mex"], check=True, capture_output=True, text=True, timeout=600)


class Gateway:
    def __init__(self, name: str):
        path = os.path.join(NATIVE, "_build", f"mex_{name}.so")
        if not os.path.exists(path):
            build()
        self.lib = C.CDLL(path)
        L = self.lib
        for fn, res, args in [("shim_struct", _P, []), ("shim_set_field", None, [_P, C.c_char_p, _P]),
                              ("shim_double", _P, [C.c_int, C.POINTER(C.c_size_t), C.POINTER(C.c_double)]),
                              ("shim_logical", _P, [C.c_int, C.POINTER(C.c_size_t), C.POINTER(C.c_ubyte)]),
                              ("shim_string", _P, [C.c_char_p]), ("shim_ndims", C.c_int, [_P]),
                              ("shim_dims", None, [_P, C.POINTER(C.c_size_t)]), ("shim_data", _P, [_P]),
                              ("shim_free", None, [_P]), ("shim_call", C.c_int, [C.c_int, C.POINTER(_P), C.c_int,
                                                                                  C.POINTER(_P)]),
                              ("shim_error", C.c_char_p, []), ("shim_log", C.c_char_p, []),
                              ("shim_clear_log", None, []), ("shim_ncalls", C.c_int, []),
                              ("shim_call_name", C.c_char_p, [C.c_int])]:
            f = getattr(L, fn)
            f.restype = res
            f.argtypes = args

    def array(self, a):
        a = np.asarray(a)
        if a.dtype == bool:
            d = np.asfortranarray(a.astype(np.uint8))
            dims = (C.c_size_t * d.ndim)(*d.shape)
            return self.lib.shim_logical(d.ndim, dims, d.ctypes.data_as(C.POINTER(C.c_ubyte)))
        d = np.asfortranarray(a, dtype=np.float64)
        if d.ndim < 2:
            d = d.reshape((1, -1) if d.ndim == 1 else (1, 1), order="F")
        dims = (C.c_size_t * d.ndim)(*d.shape)
        return self.lib.shim_double(d.ndim, dims, d.ctypes.data_as(C.POINTER(C.c_double)))

    def options(self, opts: dict):
        s = self.lib.shim_struct()
        for k, v in opts.items():
            self.lib.shim_set_field(s, k.encode(), self.lib.shim_string(v.encode()) if isinstance(v, str)
                                    else self.array(v))
        return s

    def output(self, p):
        n = self.lib.shim_ndims(p)
        dims = (C.c_size_t * n)()
        self.lib.shim_dims(p, dims)
        shape = tuple(dims)
        cnt = int(np.prod(shape))
        buf = (C.c_double * cnt).from_address(self.lib.shim_data(p))
        return np.array(np.ctypeslib.as_array(buf).reshape(shape, order="F"), order="F")

    def __call__(self, nlhs: int, *args):
        """[out1..outN] = gateway(args...); dict args become option structs."""
        prhs = (_P * len(args))(*[self.options(a) if isinstance(a, dict) else self.array(a) for a in args])
        plhs = (_P * nlhs)()
        self.lib.shim_clear_log()
        rc = self.lib.shim_call(nlhs, plhs, len(args), prhs)
        for p in prhs:
            self.lib.shim_free(p)
        if rc:
            raise RuntimeError(self.lib.shim_error().decode())
        outs = [self.output(plhs[i]) for i in range(nlhs)]
        for i in range(nlhs):
            self.lib.shim_free(plhs[i])
        return outs

    def log(self) -> str:
        return self.lib.shim_log().decode(errors="replace")

    def calls(self):
        return [self.lib.shim_call_name(i).decode() for i in range(self.lib.shim_ncalls())]
