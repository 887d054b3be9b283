"""nebula_amd — MI355X-native GO N STEPS / FIND PATH engine for Nebula Graph's traversal path.

The product is the C ABI in ``include/nbg.h`` implemented by ``nebula_amd/libnbg.so``
(host C++ + gfx950 HIP kernels).  This package is the Python host binding plus fixture
tooling (KV record builders, the RMAT generator); the nGQL front end the parity tests drive it with
is test harness (tests/support/ngql.py).
"""
from .engine import DeviceRows, Engine, LocalCluster, NbgError, comm_unique_id, nba_engine  # noqa: F401

__all__ = ["Engine", "NbgError", "DeviceRows", "LocalCluster", "comm_unique_id", "nba_engine"]
