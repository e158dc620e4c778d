"""The rank communicator of the C-ABI (capf_comm_*: RCCL over xGMI, ordered on
the session stream) and the session's device buffers, as a host without
torch.distributed (the JVM twin, DistGpuTable.scala) drives them.  A one-GPU
box runs a world of one rank: every collective is exercised end to end
(RCCL needs one GPU per rank, so wider worlds run only on a multi-GPU node;
their exchange logic is the same as dist_table.py's, covered by the gloo tests).
"""
import ctypes
from ctypes import byref, c_int32, c_int64, c_void_p

import numpy as np
import pytest

from capf_amd import _lib

pytestmark = pytest.mark.gpu


def _buf(session, nbytes):
    d = c_void_p()
    _lib.call("capf_session_alloc", session._h, int(nbytes), byref(d))
    return d


def _put(session, d, arr):
    _lib.call("capf_session_copy", session._h, d, arr.ctypes.data, arr.nbytes, 1)


def _get(session, d, arr):
    _lib.call("capf_session_copy", session._h, arr.ctypes.data, d, arr.nbytes, 2)
    return arr


def test_comm_world_of_one(gpu_session):
    s = gpu_session
    uid = (ctypes.c_uint8 * 128)()
    _lib.call("capf_comm_unique_id", uid)
    comm = c_void_p()
    _lib.call("capf_comm_init", s._h, 1, 0, uid, byref(comm))
    try:
        r, w = c_int32(), c_int32()
        _lib.call("capf_comm_rank", comm, byref(r), byref(w))
        assert (r.value, w.value) == (0, 1)
        # all-reduce SUM / MAX of int64 (the count partials; the wire-format ranges)
        vals = np.array([5, -7, 1 << 40], dtype=np.int64)
        d = _buf(s, vals.nbytes)
        _put(s, d, vals)
        _lib.call("capf_comm_all_reduce_i64", comm, d, 3, 0)
        assert _get(s, d, np.zeros(3, np.int64)).tolist() == vals.tolist()
        _lib.call("capf_comm_all_reduce_i64", comm, d, 3, 2)
        assert _get(s, d, np.zeros(3, np.int64)).tolist() == vals.tolist()
        with pytest.raises(_lib.IllegalArgumentException):
            _lib.call("capf_comm_all_reduce_i64", comm, d, 3, 1)
        # all-gather and all-to-all of packed bytes (to itself)
        msg = np.frombuffer(b"packed rows!", dtype=np.uint8).copy()
        ds, dr = _buf(s, msg.nbytes), _buf(s, msg.nbytes)
        _put(s, ds, msg)
        _lib.call("capf_comm_all_gather_bytes", comm, ds, msg.nbytes, dr)
        assert bytes(_get(s, dr, np.zeros(msg.nbytes, np.uint8))) == b"packed rows!"
        z = np.zeros(msg.nbytes, np.uint8)
        _put(s, dr, z)
        _lib.call("capf_comm_all_to_all_bytes", comm, ds, (c_int64 * 1)(msg.nbytes), dr, (c_int64 * 1)(msg.nbytes))
        assert bytes(_get(s, dr, np.zeros(msg.nbytes, np.uint8))) == b"packed rows!"
        for b in (d, ds, dr):
            _lib.call("capf_session_free", s._h, b)
        with pytest.raises(_lib.IllegalArgumentException):
            _lib.call("capf_session_free", s._h, d)
    finally:
        _lib.call("capf_comm_destroy", comm)


def test_comm_packed_shuffle_round_trip(gpu_session):
    """The shuffle a DistGpuTable runs per repartition, at world size one:
    hash route → pack rows → all-to-all → table from packed rows; the rows
    come back unchanged (as a bag) with their FOR encodings."""
    s = gpu_session
    rng = np.random.default_rng(3)
    n = 100_000
    ids = rng.integers(0, 1 << 20, n)
    fl = rng.random(n)
    t = s.table([("id", 1, ids, None), ("x", 2, fl, (rng.random(n) > 0.2).astype(np.uint8))])
    counts = (c_int64 * 1)()
    h = c_void_p()
    _lib.call("capf_table_hash_route", t._h, 1, _lib.strs(["id"]), 1, counts, byref(h))
    assert counts[0] == n
    from capf_amd.table import GpuTable
    routed = GpuTable(s, h)
    cols = ["id", "x"]
    width = (c_int32 * 2)(3, 8)
    base = (c_int64 * 2)(0, 0)
    nullable = (c_int32 * 2)(0, 1)
    W = c_int32()
    _lib.call("capf_table_pack_rows", routed._h, 2, _lib.strs(cols), width, base, nullable, byref(W), None)
    d_send, d_recv = _buf(s, n * W.value), _buf(s, n * W.value)
    _lib.call("capf_table_pack_rows", routed._h, 2, _lib.strs(cols), width, base, nullable, byref(W), d_send)
    uid = (ctypes.c_uint8 * 128)()
    _lib.call("capf_comm_unique_id", uid)
    comm = c_void_p()
    _lib.call("capf_comm_init", s._h, 1, 0, uid, byref(comm))
    try:
        nb = (c_int64 * 1)(n * W.value)
        _lib.call("capf_comm_all_to_all_bytes", comm, d_send, nb, d_recv, nb)
    finally:
        _lib.call("capf_comm_destroy", comm)
    out = c_void_p()
    _lib.call("capf_table_from_packed_rows", s._h, 2, _lib.strs(cols), (c_int32 * 2)(1, 2), width, base, nullable,
              d_recv, n, byref(out))
    back = GpuTable(s, out)
    got = sorted(zip(back.column_values("id"), back.column_values("x")), key=repr)
    want = sorted(zip(t.column_values("id"), t.column_values("x")), key=repr)
    assert got == want
    _lib.call("capf_session_free", s._h, d_send)
    _lib.call("capf_session_free", s._h, d_recv)
