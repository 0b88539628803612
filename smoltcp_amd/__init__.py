"""smoltcp_amd — MI355X-native Internet-checksum engine for smoltcp's ``wire`` checksum path.

* ``smoltcp_amd.checksum`` — ``smoltcp::wire::checksum`` scalar mirrors (C ABI, host);
* ``smoltcp_amd.phy``      — ``Checksum`` / ``ChecksumCapabilities`` policy mirrors;
* ``smoltcp_amd.engine``   — the batched HIP engine (emit / verify / data over HBM batches).

The compute lives in ``libsmolcsum.so`` (HIP kernels for gfx950 + the C ABI of
``include/smolcsum.h``).  Importing this package does not import torch.
"""
from . import checksum, phy  # noqa: F401
from ._lib import LIB_PATH, SmolError, lib  # noqa: F401
from .phy import Checksum, ChecksumCapabilities  # noqa: F401

__all__ = ["checksum", "phy", "Checksum", "ChecksumCapabilities", "SmolError", "lib", "LIB_PATH"]
