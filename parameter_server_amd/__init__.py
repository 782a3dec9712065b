"""parameter_server_amd — MI355X-native row-update apply path for Bosen-style parameter servers.

The product is libpsx.so (include/psx.h): hand-written gfx950 HIP kernels behind a
C ABI.  This package holds its ctypes binding and the host-side mirror of the
reference's server apply interface (src/petuum_ps/server/server.hpp).
"""
from . import _abi
from ._abi import PsxError, F32, F64, I32, I64, ROW_DENSE, ROW_SORTED_MAP, ROW_MAP
from .server import Server, ServerThread, TableInfo
from . import wire

__all__ = ["Server", "ServerThread", "TableInfo", "PsxError", "F32", "F64", "I32", "I64",
           "ROW_DENSE", "ROW_SORTED_MAP", "ROW_MAP", "wire"]
