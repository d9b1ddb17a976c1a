"""Host-resident record pipeline (north_star's PCIe-inclusive rate).

Records start and end in host memory (socket buffers in a server): pinned host
fragments -> hipMemcpyAsync H2D -> tlsgpu_open_batch -> hipMemcpyAsync D2H of the
plaintext, split into chunks round-robined over several HIP streams so that the
copies of one chunk overlap the kernel of another.  Descriptors stay resident
(a server keeps its descriptor ring on the device).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import DeviceBuffer, _check, open_batch


class HostPipeline:
    def __init__(self, wl, chunks: int = 32, streams: int = 4):
        self.wl = wl
        eng = wl.engine
        self.eng = eng
        lib = eng.lib
        self.streams = [eng.new_stream() for _ in range(streams)]
        self.h_body = C.c_void_p()
        self.h_out = C.c_void_p()
        _check(lib.tlsgpu_host_alloc(eng.handle, wl.body_bytes, C.byref(self.h_body)),
               "tlsgpu_host_alloc")
        _check(lib.tlsgpu_host_alloc(eng.handle, wl.pt_bytes, C.byref(self.h_out)),
               "tlsgpu_host_alloc")
        # host copy of the sealed fragments (what the NIC handed us)
        _check(lib.tlsgpu_memcpy(eng.handle, self.h_body.value, wl.d_body.ptr, wl.body_bytes,
                                 None), "tlsgpu_memcpy")
        eng.sync()
        n = wl.n
        bounds = np.linspace(0, n, chunks + 1).astype(np.int64)
        self.chunks = [(int(a), int(b)) for a, b in zip(bounds[:-1], bounds[1:]) if b > a]
        eiv = int(wl.body_off[0] % 16 and (16 - wl.body_off[0] % 16) % 16)
        self.body_lo = [int(wl.body_off[a]) for a, _ in self.chunks]
        self.body_hi = [int(wl.body_off[b - 1]) + int(wl.lengths[b - 1]) + 8 + 16 + 8
                        for _, b in self.chunks]
        self.out_lo = [int(wl.pt_off[a]) for a, _ in self.chunks]
        self.out_hi = [int(wl.pt_off[b - 1]) + int(wl.lengths[b - 1]) for _, b in self.chunks]
        del eiv

    def run(self) -> None:
        lib, eng, wl = self.eng.lib, self.eng, self.wl
        for k, (a, b) in enumerate(self.chunks):
            s = self.streams[k % len(self.streams)]
            lo, hi = self.body_lo[k], min(self.body_hi[k], wl.body_bytes)
            _check(lib.tlsgpu_memcpy(eng.handle, wl.d_body.ptr + lo, self.h_body.value + lo,
                                     hi - lo, s), "H2D")
            open_batch(wl.table, wl.d_open.ptr + 32 * a, b - a, wl.d_body.ptr, wl.d_body.nbytes,
                       wl.d_out.ptr, wl.d_out.nbytes, wl.d_status.ptr + 4 * a, s)
            olo, ohi = self.out_lo[k], self.out_hi[k]
            _check(lib.tlsgpu_memcpy(eng.handle, self.h_out.value + olo, wl.d_out.ptr + olo,
                                     ohi - olo, s), "D2H")
        for s in self.streams:
            eng.sync_stream(s)

    def host_plaintext(self, i: int) -> bytes:
        off, ln = int(self.wl.pt_off[i]), int(self.wl.lengths[i])
        return C.string_at(self.h_out.value + off, ln)

    def close(self) -> None:
        lib, eng = self.eng.lib, self.eng
        lib.tlsgpu_host_free(eng.handle, self.h_body.value)
        lib.tlsgpu_host_free(eng.handle, self.h_out.value)
        for s in self.streams:
            lib.tlsgpu_stream_destroy(eng.handle, s)
