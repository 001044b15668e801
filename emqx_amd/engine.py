"""Host-side engine over the C ABI: contexts, index snapshots, batch match and fan-out.

This is plumbing around the HIP library; every compute call runs the gfx950
kernels in libemqx_gpu_match.so.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib
from ._lib import Csr, GpuMatchError, IndexInfo, MatchStats, Opts, check, lib

BytesLike = Union[bytes, bytearray, str]


def _b(s: BytesLike) -> bytes:
    return s.encode() if isinstance(s, str) else bytes(s)


def pack(strings: Iterable[BytesLike]) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate byte strings -> (uint8 bytes padded by 64, uint64 offsets[n+1])."""
    bs = [_b(s) for s in strings]
    off = np.zeros(len(bs) + 1, np.uint64)
    if bs:
        np.cumsum([len(b) for b in bs], out=off[1:])
    data = np.frombuffer(b"".join(bs) + b"\0" * 64, np.uint8).copy()
    return data, off


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _csr_to_numpy(csr: Csr) -> Tuple[np.ndarray, np.ndarray]:
    n, nnz = csr.n_rows, csr.nnz
    ro = np.ctypeslib.as_array(csr.row_off, shape=(n + 1,)).copy()
    ids = np.ctypeslib.as_array(csr.ids, shape=(nnz,)).copy() if nnz else np.zeros(0, np.uint32)
    return ro, ids


@dataclass
class DeviceCsr:
    """A result CSR resident in HBM (owned by the library until free())."""
    ctx: "Context"
    csr: Csr

    @property
    def n_rows(self) -> int:
        return int(self.csr.n_rows)

    @property
    def nnz(self) -> int:
        return int(self.csr.nnz)

    def to_host(self) -> Tuple[np.ndarray, np.ndarray]:
        n, nnz = self.n_rows, self.nnz
        ro = np.zeros(n + 1, np.uint64)
        ids = np.zeros(max(nnz, 1), np.uint32)
        self.ctx.memcpy_d2h(ro, C.cast(self.csr.row_off, C.c_void_p).value, (n + 1) * 8)
        if nnz:
            self.ctx.memcpy_d2h(ids, C.cast(self.csr.ids, C.c_void_p).value, nnz * 4)
        return ro, ids[:nnz]

    def rows(self, start: int, count: int) -> Tuple[np.ndarray, np.ndarray]:
        """Rows [start, start+count) copied to the host: (row offsets rebased to 0, ids)."""
        ro = np.zeros(count + 1, np.uint64)
        self.ctx.memcpy_d2h(ro, C.cast(self.csr.row_off, C.c_void_p).value + 8 * start, (count + 1) * 8)
        nnz = int(ro[-1] - ro[0])
        ids = np.zeros(max(nnz, 1), np.uint32)
        if nnz:
            self.ctx.memcpy_d2h(ids, C.cast(self.csr.ids, C.c_void_p).value + 4 * int(ro[0]), nnz * 4)
        return ro - ro[0], ids[:nnz]

    def free(self):
        if self.csr.row_off or self.csr.ids:
            check(lib().emqx_gm_csr_free(self.ctx.h, C.byref(self.csr)), self.ctx.h, "csr_free")

    def __del__(self):
        try:
            if self.ctx.h:
                self.free()
        except Exception:
            pass


class PendingMatch:
    """A submitted match call (emqx_gm_match_submit); wait() exactly once."""

    def __init__(self, ctx: "Context", call):
        self.ctx, self.call = ctx, call

    def wait(self) -> "DeviceCsr":
        if not self.call:
            raise GpuMatchError(_lib.EINVAL, "match_wait: already waited")
        csr = Csr()
        call, self.call = self.call, None
        check(lib().emqx_gm_match_wait(self.ctx.h, call, C.byref(csr)), self.ctx.h, "match_wait")
        return DeviceCsr(self.ctx, csr)

    def __del__(self):
        try:
            if self.call and self.ctx.h:
                self.wait().free()
        except Exception:
            pass


class HostCsr:
    """A result CSR in host memory owned by the library (emqx_gm_match without
    DEVICE_IO); ``row_off`` / ``ids`` are views valid until ``free()``."""

    def __init__(self, ctx: "Context", csr: Csr):
        self.ctx, self.csr = ctx, csr
        n, nnz = int(csr.n_rows), int(csr.nnz)
        self.row_off = np.ctypeslib.as_array(csr.row_off, shape=(n + 1,))
        self.ids = np.ctypeslib.as_array(csr.ids, shape=(nnz,)) if nnz else np.zeros(0, np.uint32)

    @property
    def nnz(self) -> int:
        return int(self.csr.nnz)

    def free(self):
        if self.csr.row_off or self.csr.ids:
            self.row_off = self.ids = None
            lib().emqx_gm_csr_free(self.ctx.h, C.byref(self.csr))


class Index:
    """An immutable, reference-counted index snapshot resident in HBM."""

    def __init__(self, ctx: "Context", handle, perm: np.ndarray):
        self.ctx = ctx
        self.h = handle
        self.perm = perm

    @property
    def info(self) -> IndexInfo:
        inf = IndexInfo()
        check(lib().emqx_gm_index_info(self.h, C.byref(inf)), None, "index_info")
        return inf

    @property
    def n_filters(self) -> int:
        return int(self.info.n_filters)

    def empty(self) -> bool:
        """emqx_trie:empty/0: the index holds no wildcard filter."""
        return bool(self.info.trie_empty)

    def filter(self, fid: int) -> bytes:
        p, n = C.c_void_p(), C.c_uint64()
        check(lib().emqx_gm_index_filter(self.h, fid, C.byref(p), C.byref(n)), None, "index_filter")
        return C.string_at(p, n.value) if n.value else b""

    def subscriber_count(self, fid: int) -> int:
        """Length of filter ``fid``'s segment in a fan-out row (emqx_gm_index_subscriber_count)."""
        n = C.c_uint64()
        check(lib().emqx_gm_index_subscriber_count(self.h, fid, C.byref(n)), None, "index_subscriber_count")
        return int(n.value)

    def filters(self) -> List[bytes]:
        return [self.filter(i) for i in range(self.n_filters)]

    def export_size(self, with_blob: bool = True) -> int:
        n = C.c_uint64()
        check(lib().emqx_gm_index_export(self.ctx.h, self.h, 0 if with_blob else _lib.IMAGE_NO_BLOB, None,
                                         C.byref(n)), self.ctx.h, "index_export")
        return int(n.value)

    def export(self, with_blob: bool = True, out: Optional[np.ndarray] = None) -> np.ndarray:
        """The snapshot as a host image (emqx_gm_index_export): the host tables
        and, with ``with_blob``, the device tables.  ``out`` (uint8, e.g. a
        shared-memory map) receives it when given and large enough."""
        flags = 0 if with_blob else _lib.IMAGE_NO_BLOB
        n = C.c_uint64()
        check(lib().emqx_gm_index_export(self.ctx.h, self.h, flags, None, C.byref(n)), self.ctx.h, "index_export")
        buf = out if out is not None and out.nbytes >= n.value else np.empty(n.value, np.uint8)
        check(lib().emqx_gm_index_export(self.ctx.h, self.h, flags, _ptr(buf), C.byref(n)), self.ctx.h,
              "index_export")
        return buf[:n.value]

    def device_blob(self) -> Tuple[int, int]:
        """(device pointer, bytes) of the snapshot's device tables (emqx_gm_index_device_blob)."""
        p, n = C.c_void_p(), C.c_uint64()
        check(lib().emqx_gm_index_device_blob(self.h, C.byref(p), C.byref(n)), None, "index_device_blob")
        return p.value, int(n.value)

    def replica_digest(self, k: int) -> Tuple[int, int]:
        """(tables, subscriber CSR) FNV digests of replica k of this snapshot
        (0: the snapshot itself; k: its replica on the context's k-th member)."""
        t, u = C.c_uint64(), C.c_uint64()
        check(lib().emqx_gm_index_replica_digest(self.ctx.h, self.h, k, C.byref(t), C.byref(u)), self.ctx.h,
              "index_replica_digest")
        return int(t.value), int(u.value)

    def release(self):
        if self.h:
            lib().emqx_gm_index_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


def _init_torch_runtime():
    """torch's HIP runtime must come up before the library's when both live in
    one process (a library-first process leaves torch with "No HIP
    GPUs are available").  So a context initialises torch's device runtime
    first whenever torch is importable; a process without torch is unaffected."""
    try:
        import torch
    except Exception:  # (no torch: nothing to order)
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


class Context:
    """A context binds one HIP device (one process per GPU), or -- with
    ``devices`` -- a list of them: every index is then replicated to each
    listed device and a host-buffer match spreads its batch over all of them
    (emqx_gm_opts.n_devices)."""

    def __init__(self, device: int = 0, mirror: Optional[str] = None, devices: Optional[Sequence[int]] = None):
        """``mirror``: None (library default: the host copy of a plain index's
        tables is kept from the build up to 8 GiB, loaded on the first update
        above), "eager" or "lazy" (EMQX_GM_OPEN_MIRROR_*).  ``devices``: the
        device list of a multi-device context (repeats allowed: replicas on one
        device)."""
        _init_torch_runtime()
        o = Opts()
        o.device = device
        o.flags = {None: 0, "eager": _lib.OPEN_MIRROR_EAGER, "lazy": _lib.OPEN_MIRROR_LAZY}[mirror]
        if devices is not None:
            devices = list(devices)
            if not 1 <= len(devices) <= _lib.MAX_DEVICES:
                raise ValueError(f"1..{_lib.MAX_DEVICES} devices")
            o.n_devices = len(devices)
            for k, d in enumerate(devices):
                o.devices[k] = d
            device = devices[0]
        h = C.c_void_p()
        rc = lib().emqx_gm_open(C.byref(o), C.byref(h))
        if rc != _lib.OK:
            raise GpuMatchError(rc, f"emqx_gm_open(devices={devices if devices else [device]}) failed "
                                    f"(no MI355X visible?)")
        self.h = h
        self.device = device
        self._stats_buf = MatchStats()

    @property
    def devices(self) -> List[int]:
        n = C.c_uint32()
        check(lib().emqx_gm_devices(self.h, None, C.byref(n)), self.h, "devices")
        arr = (C.c_int32 * n.value)()
        check(lib().emqx_gm_devices(self.h, arr, C.byref(n)), self.h, "devices")
        return list(arr)

    def host_alloc(self, nbytes: int) -> np.ndarray:
        """A page-locked uint8 buffer (emqx_gm_host_alloc): topics packed into it
        cross PCIe by DMA without a staging copy.  Free with host_free()."""
        p = C.c_void_p()
        check(lib().emqx_gm_host_alloc(self.h, nbytes, C.byref(p)), self.h, "host_alloc")
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(max(nbytes, 1),))[:nbytes]

    def host_free(self, buf: np.ndarray):
        check(lib().emqx_gm_host_free(self.h, C.c_void_p(buf.ctypes.data)), self.h, "host_free")

    def close(self):
        if self.h:
            lib().emqx_gm_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------------ index
    def build_index(self, filters, subs=None, _entry: str = "emqx_gm_index_build") -> Index:
        """filters: sequence of bytes/str, or a packed (bytes, offsets) pair.
        subs: optional per-filter subscriber lists, or a packed (offsets, ids) pair."""
        fb, fo = filters if isinstance(filters, tuple) else pack(filters)
        n = len(fo) - 1
        so = si = None
        if subs is not None:
            if isinstance(subs, tuple):
                so = np.ascontiguousarray(subs[0], np.uint64)
                si = np.ascontiguousarray(subs[1], np.uint32)
            else:
                so = np.zeros(n + 1, np.uint64)
                np.cumsum([len(s) for s in subs], out=so[1:])
                si = np.fromiter((x for s in subs for x in s), np.uint32, count=int(so[-1]))
            if len(si) == 0:
                si = np.zeros(1, np.uint32)
        perm = np.zeros(max(n, 1), np.uint32)
        h = C.c_void_p()
        check(getattr(lib(), _entry)(self.h, _ptr(fb), _ptr(fo), n, _ptr(so), _ptr(si), _ptr(perm), C.byref(h)),
              self.h, _entry[8:])
        return Index(self, h, perm[:n])

    def build_index_sharded(self, filters, subs=None) -> Index:
        """A prefix-sharded index over this context's devices (emqx_gm_index_build_sharded):
        one shard per listed device, each topic matched on its one shard."""
        return self.build_index(filters, subs, _entry="emqx_gm_index_build_sharded")

    def import_index(self, image: np.ndarray, d_blob: Optional[int] = None) -> Index:
        """A snapshot from an image (emqx_gm_index_import); its device tables from
        the image or, with ``d_blob``, copied from that device pointer."""
        img = np.ascontiguousarray(image, np.uint8)
        h = C.c_void_p()
        check(lib().emqx_gm_index_import(self.h, _ptr(img), img.nbytes, C.c_void_p(d_blob) if d_blob else None,
                                         C.byref(h)), self.h, "index_import")
        return Index(self, h, np.zeros(0, np.uint32))

    def build_index_shard(self, filters, global_ids: np.ndarray, subs=None) -> Index:
        """An index over one shard whose rows carry ``global_ids`` (emqx_gm_index_build_shard)."""
        fb, fo = filters if isinstance(filters, tuple) else pack(filters)
        n = len(fo) - 1
        g = np.ascontiguousarray(global_ids, np.uint32)
        if len(g) != n:
            raise ValueError("one global id per filter")
        perm = np.zeros(max(n, 1), np.uint32)
        h = C.c_void_p()
        check(lib().emqx_gm_index_build_shard(self.h, _ptr(fb), _ptr(fo), n, _ptr(g) if n else None, None, None,
                                              _ptr(perm), C.byref(h)), self.h, "index_build_shard")
        return Index(self, h, perm[:n])

    def update_index(self, index: Index, ops) -> Index:
        """A new snapshot = ``index`` with ``ops`` applied in order; ops is a
        sequence of (filter, insert: bool).  ``index`` stays valid (RCU)."""
        ops = list(ops)
        fb, fo = pack([f for f, _ in ops])
        kinds = np.array([1 if ins else 0 for _, ins in ops] or [0], np.uint8)
        h = C.c_void_p()
        check(lib().emqx_gm_index_update(self.h, index.h, _ptr(fb), _ptr(fo), _ptr(kinds), len(ops), C.byref(h)),
              self.h, "index_update")
        return Index(self, h, np.zeros(0, np.uint32))

    SUB_OPS = {"unsubscribe": 0, "subscribe": 1, "route_add": 2, "route_delete": 3}

    def update_subs(self, index: Index, ops) -> Index:
        """A new snapshot of an index built with subscriber lists, with ``ops``
        applied in order: (filter, subscriber id, op) with op True/"subscribe",
        False/"unsubscribe", or "route_add"/"route_delete" (the filter is routed to
        another destination: it stays in the index without a local subscriber) --
        a filter's first holder adds its route, the last one leaving deletes it
        (emqx_gm_index_update_subs).  ``index`` stays valid (RCU)."""
        ops = list(ops)
        fb, fo = pack([f for f, _, _ in ops])
        subs = np.array([s for _, s, _ in ops] or [0], np.uint32)
        kinds = np.array([(1 if k else 0) if isinstance(k, bool) else self.SUB_OPS[k] for _, _, k in ops] or [0],
                         np.uint8)
        h = C.c_void_p()
        check(lib().emqx_gm_index_update_subs(self.h, index.h, _ptr(fb), _ptr(fo), _ptr(subs), _ptr(kinds), len(ops),
                                              C.byref(h)), self.h, "index_update_subs")
        return Index(self, h, np.zeros(0, np.uint32))

    # ------------------------------------------------------------------ match
    def match(self, index: Index, topics, exact: bool = True) -> Tuple[np.ndarray, np.ndarray]:
        """Batch emqx_router:match_routes/1 (exact=True) or emqx_trie:match/1
        (exact=False).  Returns CSR (row_off uint64[n+1], filter ids uint32)."""
        tb, to = topics if isinstance(topics, tuple) else pack(topics)
        csr = Csr()
        flags = _lib.WITH_EXACT if exact else 0
        check(lib().emqx_gm_match(self.h, index.h, _ptr(tb), _ptr(to), len(to) - 1, flags, C.byref(csr)),
              self.h, "match")
        try:
            return _csr_to_numpy(csr)
        finally:
            lib().emqx_gm_csr_free(self.h, C.byref(csr))

    def match_host(self, index: Index, topics, exact: bool = True) -> "HostCsr":
        """Host buffers in, host rows out (the NIF's call), without copying the
        result: numpy views of the library's buffers, valid until ``free()``."""
        tb, to = topics if isinstance(topics, tuple) else pack(topics)
        csr = Csr()
        flags = _lib.WITH_EXACT if exact else 0
        check(lib().emqx_gm_match(self.h, index.h, _ptr(tb), _ptr(to), len(to) - 1, flags, C.byref(csr)),
              self.h, "match")
        return HostCsr(self, csr)

    def match_device(self, index: Index, d_bytes: int, d_off: int, n: int, exact: bool = True) -> DeviceCsr:
        """Inputs already in HBM (device pointers); the result stays in HBM."""
        csr = Csr()
        flags = _lib.DEVICE_IO | (_lib.WITH_EXACT if exact else 0)
        check(lib().emqx_gm_match(self.h, index.h, C.c_void_p(d_bytes), C.c_void_p(d_off), n, flags,
                                  C.byref(csr)), self.h, "match")
        return DeviceCsr(self, csr)

    def match_submit(self, index: Index, d_bytes: int, d_off: int, n: int, exact: bool = True,
                     timed: bool = True) -> "PendingMatch":
        """emqx_gm_match_submit: the call's kernels queued on the device, no wait;
        ``wait()`` on the result gives the DeviceCsr.  Inputs stay the caller's until then.
        ``timed`` False: EMQX_GM_NO_TIMING (no main-pass timestamps on the stream)."""
        call = C.c_void_p()
        flags = _lib.DEVICE_IO | (_lib.WITH_EXACT if exact else 0) | (0 if timed else _lib.NO_TIMING)
        check(lib().emqx_gm_match_submit(self.h, index.h, C.c_void_p(d_bytes), C.c_void_p(d_off), n, flags,
                                         C.byref(call)), self.h, "match_submit")
        return PendingMatch(self, call)

    def fanout(self, index: Index, row_off: np.ndarray, ids: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """emqx_broker:dispatch/2 over each row's matched filters -> subscriber CSR (multiset rows)."""
        ro = np.ascontiguousarray(row_off, np.uint64)
        ii = np.ascontiguousarray(ids, np.uint32)
        if len(ii) == 0:
            ii = np.zeros(1, np.uint32)
        m = Csr()
        m.n_rows = len(ro) - 1
        m.nnz = int(ro[-1])
        m.row_off = ro.ctypes.data_as(C.POINTER(C.c_uint64))
        m.ids = ii.ctypes.data_as(C.POINTER(C.c_uint32))
        m.on_device = 0
        out = Csr()
        check(lib().emqx_gm_fanout(self.h, index.h, C.byref(m), 0, C.byref(out)), self.h, "fanout")
        try:
            return _csr_to_numpy(out)
        finally:
            lib().emqx_gm_csr_free(self.h, C.byref(out))

    def match_fanout(self, index: Index, topics, exact: bool = True):
        """emqx_broker:publish/1's route + dispatch of a batch in one call
        (emqx_gm_match_fanout): ((row_off, filter ids), (row_off, subscriber ids)),
        equal to match() followed by fanout() -- one device round trip for a
        publish window."""
        tb, to = topics if isinstance(topics, tuple) else pack(topics)
        m, d = Csr(), Csr()
        flags = _lib.WITH_EXACT if exact else 0
        check(lib().emqx_gm_match_fanout(self.h, index.h, _ptr(tb), _ptr(to), len(to) - 1, flags, C.byref(m),
                                         C.byref(d)), self.h, "match_fanout")
        try:
            return _csr_to_numpy(m), _csr_to_numpy(d)
        finally:
            lib().emqx_gm_csr_free(self.h, C.byref(m))
            lib().emqx_gm_csr_free(self.h, C.byref(d))

    def fanout_part(self, index: Index, matches: DeviceCsr, part: int, n_parts: int) -> Tuple[DeviceCsr, int]:
        """Part ``part`` of ``n_parts`` of the fan-out of ``matches`` (emqx_gm_fanout_part):
        a device CSR whose row_off are the global delivery offsets and whose ids are the
        contiguous delivery range starting at the returned global number."""
        out = Csr()
        first = C.c_uint64()
        check(lib().emqx_gm_fanout_part(self.h, index.h, C.byref(matches.csr), part, n_parts, _lib.DEVICE_IO,
                                        C.byref(out), C.byref(first)), self.h, "fanout_part")
        return DeviceCsr(self, out), int(first.value)

    def fanout_device(self, index: Index, matches: DeviceCsr) -> DeviceCsr:
        out = Csr()
        check(lib().emqx_gm_fanout(self.h, index.h, C.byref(matches.csr), _lib.DEVICE_IO, C.byref(out)),
              self.h, "fanout")
        return DeviceCsr(self, out)

    # ------------------------------------------------------------------ sharded rows
    def csr_row_lengths(self, res: DeviceCsr, d_out: int):
        """Row lengths (u32) of a device CSR into device memory at ``d_out``."""
        check(lib().emqx_gm_csr_row_lengths(self.h, C.byref(res.csr), C.c_void_p(d_out)), self.h, "csr_row_lengths")

    def offsets_lengths(self, d_off: int, n: int, d_out: int):
        """Lengths (u32) of n device segments given by u64 offsets d_off[0..n] into
        ``d_out`` (emqx_gm_csr_row_lengths over a CSR whose row offsets are d_off)."""
        if not n:
            return
        c = Csr()
        c.n_rows, c.nnz, c.on_device = n, 0, 1
        c.row_off = C.cast(C.c_void_p(d_off), C.POINTER(C.c_uint64))
        check(lib().emqx_gm_csr_row_lengths(self.h, C.byref(c), C.c_void_p(d_out)), self.h, "csr_row_lengths")

    def merge_rows(self, n_rows: int, stride: int, pieces: int, d_lens: int, d_ids: int) -> DeviceCsr:
        """Merge per-shard rows by global id (emqx_gm_merge_rows); result stays on the device."""
        out = Csr()
        check(lib().emqx_gm_merge_rows(self.h, n_rows, stride, pieces, C.c_void_p(d_lens), C.c_void_p(d_ids),
                                       _lib.DEVICE_IO, C.byref(out)), self.h, "merge_rows")
        return DeviceCsr(self, out)

    def route_topics(self, route: "Route", d_tb: int, d_to: int, n: int, d_dest: int):
        """emqx_gm_route_topics: the shard of each device topic into d_dest (u32)."""
        check(lib().emqx_gm_route_topics(self.h, route.h, C.c_void_p(d_tb), C.c_void_p(d_to), n,
                                         C.c_void_p(d_dest)), self.h, "route_topics")

    def route_partition(self, route: "Route", d_tb: int, d_to: int, n: int, d_perm: int, d_plen: int, d_split: int):
        """emqx_gm_route_partition: the batch's send order by shard (u32 perm and
        lengths, n each) and the topics / bytes per shard (u64 pairs)."""
        check(lib().emqx_gm_route_partition(self.h, route.h, C.c_void_p(d_tb), C.c_void_p(d_to), n,
                                            C.c_void_p(d_perm), C.c_void_p(d_plen), C.c_void_p(d_split)),
              self.h, "route_partition")

    def permute_topics(self, d_tb: int, d_to: int, n: int, d_perm: int, d_out: int, d_out_off: int):
        check(lib().emqx_gm_permute_topics(self.h, C.c_void_p(d_tb), C.c_void_p(d_to), n, C.c_void_p(d_perm),
                                           C.c_void_p(d_out), C.c_void_p(d_out_off)), self.h, "permute_topics")

    def unpermute_rows(self, n: int, d_perm: int, d_lens: int, d_ids: int) -> DeviceCsr:
        out = Csr()
        check(lib().emqx_gm_unpermute_rows(self.h, n, C.c_void_p(d_perm), C.c_void_p(d_lens), C.c_void_p(d_ids),
                                           _lib.DEVICE_IO, C.byref(out)), self.h, "unpermute_rows")
        return DeviceCsr(self, out)

    def memcpy_d2d(self, dst_ptr: int, src_ptr: int, nbytes: int):
        if nbytes:
            check(lib().emqx_gm_memcpy(self.h, C.c_void_p(dst_ptr), C.c_void_p(src_ptr), nbytes, 2), self.h, "memcpy")

    # ------------------------------------------------------------------ misc
    def stats(self) -> dict:
        s = MatchStats()
        check(lib().emqx_gm_last_stats(self.h, C.byref(s)), self.h, "last_stats")
        return {k: getattr(s, k) for k, _ in MatchStats._fields_}

    def update_stats(self) -> dict:
        """What this thread's last index call (build, import, update, update_subs) did
        (emqx_gm_last_update_stats): path, replica mode, mirror download, times."""
        s = _lib.UpdateStats()
        check(lib().emqx_gm_last_update_stats(self.h, C.byref(s)), self.h, "last_update_stats")
        d = {k: getattr(s, k) for k, _ in _lib.UpdateStats._fields_}
        d["kind"] = _lib.UPD_KINDS.get(d["kind"], d["kind"])
        d["replica_mode"] = _lib.REP_MODES.get(d["replica_mode"], d["replica_mode"])
        d["mirror_loaded"] = bool(d["mirror_loaded"])
        return d

    def last_kernel_ms(self) -> float:
        """stats()["match_kernel_ms"] without building the dict (a serving loop's per-call read)."""
        s = self._stats_buf
        check(lib().emqx_gm_last_stats(self.h, C.byref(s)), self.h, "last_stats")
        return s.match_kernel_ms

    def synchronize(self):
        check(lib().emqx_gm_synchronize(self.h), self.h, "synchronize")

    def set_stream(self, hip_stream: int):
        check(lib().emqx_gm_set_stream(self.h, C.c_void_p(hip_stream or None)), self.h, "set_stream")

    def memcpy_d2h(self, dst: np.ndarray, src_ptr: int, nbytes: int):
        check(lib().emqx_gm_memcpy(self.h, _ptr(dst), C.c_void_p(src_ptr), nbytes, 1), self.h, "memcpy")

    def memcpy_h2d(self, dst_ptr: int, src: np.ndarray, nbytes: int):
        check(lib().emqx_gm_memcpy(self.h, C.c_void_p(dst_ptr), _ptr(src), nbytes, 0), self.h, "memcpy")

    def dev_alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        check(lib().emqx_gm_dev_alloc(self.h, nbytes, C.byref(p)), self.h, "dev_alloc")
        return p.value

    def dev_free(self, ptr: int):
        lib().emqx_gm_dev_free(self.h, C.c_void_p(ptr))

    def pool_trim(self):
        lib().emqx_gm_pool_trim(self.h)

    def matched_filter_bytes(self, index: Index, res: DeviceCsr) -> int:
        out = C.c_uint64()
        check(lib().emqx_gm_matched_filter_bytes(self.h, index.h, C.byref(res.csr), C.byref(out)), self.h,
              "matched_filter_bytes")
        return int(out.value)

    def gen_topics_device(self, filter_codes: np.ndarray, seed: int, start: int, n: int) -> Tuple[int, int, int]:
        """Generate topics [start, start+n) of the §8d workload on the device.
        Returns (d_bytes, d_off, total_bytes); free both with dev_free."""
        fc = np.ascontiguousarray(filter_codes, np.int16)
        db, do, tot = C.c_void_p(), C.c_void_p(), C.c_uint64()
        check(lib().emqx_gm_gen_topics(self.h, _ptr(fc) if len(fc) else None, len(fc), seed, start, n,
                                       C.byref(db), C.byref(do), C.byref(tot)), self.h, "gen_topics")
        return db.value, do.value, int(tot.value)


# ---------------------------------------------------------------------- sharding helpers (host)
def filter_ranks(fb: np.ndarray, fo: np.ndarray) -> Tuple[np.ndarray, int]:
    """Global id of each filter = its rank among the unique filters (emqx_gm_filter_ranks)."""
    n = len(fo) - 1
    out = np.zeros(max(n, 1), np.uint32)
    nu = C.c_uint64()
    check(lib().emqx_gm_filter_ranks(_ptr(fb), _ptr(fo), n, _ptr(out), C.byref(nu)), None, "filter_ranks")
    return out[:n], int(nu.value)


def shard_of(fb: np.ndarray, fo: np.ndarray, n_shards: int) -> np.ndarray:
    n = len(fo) - 1
    out = np.zeros(max(n, 1), np.uint32)
    check(lib().emqx_gm_shard_of(_ptr(fb), _ptr(fo), n, n_shards, _ptr(out)), None, "shard_of")
    return out[:n]


def select_filters(fb: np.ndarray, fo: np.ndarray, shard: np.ndarray, want: int) -> Tuple[np.ndarray, np.ndarray]:
    """The filters with shard == want, packed like pack()."""
    n = len(fo) - 1
    sh = np.ascontiguousarray(shard, np.uint32)
    k, nb = C.c_uint64(), C.c_uint64()
    check(lib().emqx_gm_select_filters(_ptr(fb), _ptr(fo), n, _ptr(sh), want, None, None, C.byref(k), C.byref(nb)),
          None, "select_filters")
    ob = np.zeros(nb.value + 64, np.uint8)
    oo = np.zeros(k.value + 1, np.uint64)
    check(lib().emqx_gm_select_filters(_ptr(fb), _ptr(fo), n, _ptr(sh), want, _ptr(ob), _ptr(oo), C.byref(k),
                                       C.byref(nb)), None, "select_filters")
    return ob, oo


ALL_SHARDS = 0xFFFFFFFF


class Route:
    """The topic -> shard map of a prefix-sharded filter set (emqx_gm_prefix_plan)."""

    def __init__(self, h, n_shards: int):
        self.h, self.n_shards = h, n_shards

    def route_host(self, tb: np.ndarray, to: np.ndarray) -> np.ndarray:
        n = len(to) - 1
        out = np.zeros(max(n, 1), np.uint32)
        check(lib().emqx_gm_route_topics_host(self.h, _ptr(tb), _ptr(to), n, _ptr(out)), None, "route_topics_host")
        return out[:n]

    def release(self):
        if self.h:
            lib().emqx_gm_route_release(self.h)
            self.h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


def prefix_plan(fb: np.ndarray, fo: np.ndarray, n_shards: int) -> Tuple[np.ndarray, "Route"]:
    """Prefix sharding (emqx_gm_prefix_plan): each filter's shard (ALL_SHARDS:
    every shard) and the topic route."""
    n = len(fo) - 1
    out = np.zeros(max(n, 1), np.uint32)
    h = C.c_void_p()
    check(lib().emqx_gm_prefix_plan(_ptr(fb), _ptr(fo), n, n_shards, _ptr(out), C.byref(h)), None, "prefix_plan")
    return out[:n], Route(h, n_shards)


# ---------------------------------------------------------------------- workload
def gen_filter_codes(seed: int, n: int, wildcard_only: bool = False) -> np.ndarray:
    out = np.zeros((n, 5), np.int16)
    check(lib().emqx_gm_gen_filter_codes(seed, n, int(wildcard_only), _ptr(out)), None, "gen_filter_codes")
    return out


def render_codes(codes: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    codes = np.ascontiguousarray(codes, np.int16)
    n = len(codes)
    off = np.zeros(n + 1, np.uint64)
    total = lib().emqx_gm_render_codes(_ptr(codes), n, None, _ptr(off))
    data = np.zeros(int(total) + 64, np.uint8)
    lib().emqx_gm_render_codes(_ptr(codes), n, _ptr(data), _ptr(off))
    return data, off
