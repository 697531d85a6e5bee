"""GQMAP_POLICY="name=value,..." for the profiling scripts: sets the
library's execution policies (gqmap_debug_policy) before any context is
created.  The library itself reads no environment variables."""
import os


def apply():
    spec = os.environ.get("GQMAP_POLICY", "")
    if not spec:
        return
    from gqmap_opticalflow_amd import _lib
    for item in spec.split(","):
        name, _, value = item.partition("=")
        _lib.debug_policy(name.strip(), int(value))
