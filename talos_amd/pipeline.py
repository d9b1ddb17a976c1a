"""Host-resident record pipeline (north_star's PCIe-inclusive rate).

Records start and end in host memory (socket buffers in a server): the engine's
``tlsgpu_open_host`` takes pinned host descriptors and fragments, mirrors them in
HBM chunk by chunk over several HIP streams (H2D of one chunk and D2H of another
overlap the kernels of a third) and returns plaintext and statuses in host
memory.  This module only allocates the pinned buffers and calls it.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import RECORD_DTYPE, _check, open_host


class HostPipeline:
    """A Workload's open batch as the host would hold it: fragments, descriptors
    and statuses in pinned host memory (copied once from the device workload)."""

    def __init__(self, wl):
        self.wl = wl
        eng = wl.engine
        self.eng = eng
        lib = eng.lib
        self.bufs = []

        def pinned(nbytes):
            p = C.c_void_p()
            _check(lib.tlsgpu_host_alloc(eng.handle, nbytes, C.byref(p)), "tlsgpu_host_alloc")
            self.bufs.append(p.value)
            return p.value

        self.h_body = pinned(wl.body_bytes)
        self.h_out = pinned(wl.pt_bytes)
        self.h_recs = pinned(32 * wl.n)
        self.h_status = pinned(4 * wl.n)
        # the sealed fragments as the NIC handed them over, and the descriptors
        _check(lib.tlsgpu_memcpy(eng.handle, self.h_body, wl.d_body.ptr, wl.body_bytes, None),
               "tlsgpu_memcpy")
        _check(lib.tlsgpu_memcpy(eng.handle, self.h_recs, wl.d_open.ptr, 32 * wl.n, None),
               "tlsgpu_memcpy")
        eng.sync()

    def run(self) -> None:
        wl = self.wl
        open_host(wl.table, self.h_recs, wl.n, self.h_body, wl.body_bytes, self.h_out,
                  wl.pt_bytes, self.h_status)

    def status(self) -> np.ndarray:
        return np.ctypeslib.as_array((C.c_int32 * self.wl.n).from_address(self.h_status)).copy()

    def host_plaintext(self, i: int) -> bytes:
        off, ln = int(self.wl.pt_off[i]), int(self.wl.lengths[i])
        return C.string_at(self.h_out + off, ln)

    def close(self) -> None:
        for p in self.bufs:
            self.eng.lib.tlsgpu_host_free(self.eng.handle, p)
        self.bufs = []


assert RECORD_DTYPE.itemsize == 32
