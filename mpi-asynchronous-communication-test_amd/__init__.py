"""MI355X-native aggregator exchange (all-to-many / many-to-all), the hot path of
QiaoK/MPI-Asynchronous-Communication-Test's ./test, methods 1-12.

Native parts: lib/libxghost.so (schedules, C), lib/libxg.so (HIP kernels +
RCCL), bin/test (drop-in CLI).  This Python package is the ctypes harness used
by bench.py and the tests.
"""
from . import xg  # noqa: F401
