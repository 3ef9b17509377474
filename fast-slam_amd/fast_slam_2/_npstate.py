"""numpy's global legacy RandomState read and written in place, for the drop-in
iterate() (numpy's own stream, fs2_mt_draw).

np.random.get_state() / set_state() cost ~40-70 us each: numpy's MT19937.state
property copies the 624-word key into a new array one element at a time.  The
drop-in calls both once per scan (reference fast_slam_2.py:79,81,183 consume
numpy's stream), about a fifth of a scan at config 3.  This view moves the same
fields with two memmoves instead:

- key[624] and pos: MT19937's C state (numpy's mt19937_state: uint32 key[624];
  int pos), at MT19937.ctypes.state_address -- the same layout as the first 2500
  bytes of include/fs2.h's fs2_mt_state;
- has_gauss and gauss: RandomState's aug_bitgen_t {bitgen_t *bit_generator;
  int has_gauss; double gauss}, the field after the RandomState's bitgen_t
  {void *state; 4 function pointers} (numpy/random/mtrand.pyx; the Cython
  object starts with PyObject_HEAD, its vtable and _bit_generator pointers).

The layout is not assumed, it is proven before use: the RandomState's bitgen_t
must hold the MT19937's state address and the aug_bitgen_t must point back at
that bitgen_t (two pointer identities), and a round trip through numpy's own
get_state / set_state (a cached gauss set by numpy, read here; written here, read
by numpy) must agree.  Anything else -- another numpy, another bit generator, a
debug build -- and `view()` returns None: the caller uses get_state / set_state.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

_PTR = C.sizeof(C.c_void_p)
_STATE_BYTES = 624 * 4 + 4            # key[624], pos


class LegacyStateView:
    def __init__(self):
        rs = np.random.mtrand._rand
        bg = rs._bit_generator
        if type(bg).__name__ != "MT19937":
            raise TypeError("not MT19937")
        base = id(rs)
        head = C.sizeof(C.c_ssize_t) + _PTR              # PyObject_HEAD (refcount, type)

        def ptr(off):
            return C.c_void_p.from_address(base + off).value

        # bitgen_t {state, 4 function pointers} follows the vtable and _bit_generator
        # pointers; aug_bitgen_t follows it and points back at it
        bitgen = None
        for off in range(head, head + 4 * _PTR, _PTR):
            if ptr(off) == bg.ctypes.state_address and ptr(off + 5 * _PTR) == base + off:
                bitgen = off
                break
        if bitgen is None:
            raise TypeError("RandomState layout not recognised")
        aug = bitgen + 5 * _PTR
        self._rs = rs
        self._bg = bg                                    # keeps the state's owner alive
        self._state = bg.ctypes.state_address
        self._hg = C.c_int.from_address(base + aug + _PTR)
        self._g = C.c_double.from_address(base + aug + 2 * _PTR)
        self._check()

    def _check(self):
        saved = np.random.get_state()
        try:
            _, key, pos, _, _ = saved
            np.random.set_state(("MT19937", key, pos, 1, 0.1234567890123))
            probe = _Probe()
            self.read(probe)
            ok = (probe.has_gauss == 1 and probe.gauss == 0.1234567890123 and probe.pos == pos
                  and np.array_equal(np.frombuffer(bytes(probe.key), np.uint32), key))
            probe.has_gauss, probe.gauss = 0, 0.0
            probe.pos = (int(pos) + 1) % 625
            self.write(probe)
            st = np.random.get_state()
            ok = ok and st[3] == 0 and st[4] == 0.0 and st[2] == probe.pos and np.array_equal(st[1], key)
        finally:
            np.random.set_state(saved)
        if not ok:
            raise TypeError("RandomState round trip disagrees")

    def alive(self) -> bool:
        """Still numpy's global RandomState (np.random.seed / set_state keep it)."""
        return np.random.mtrand._rand is self._rs and self._rs._bit_generator is self._bg

    def read(self, out):
        """numpy's state into an fs2_mt_state (key, pos, has_gauss, gauss)."""
        C.memmove(C.addressof(out), self._state, _STATE_BYTES)
        out.has_gauss = self._hg.value
        out.gauss = self._g.value

    def write(self, st):
        """An fs2_mt_state into numpy's state (what set_state does for MT19937)."""
        C.memmove(self._state, C.addressof(st), _STATE_BYTES)
        self._hg.value = int(st.has_gauss)
        self._g.value = float(st.gauss)


class _Probe(C.Structure):            # fs2_mt_state's layout (include/fs2.h)
    _fields_ = [("key", C.c_uint32 * 624), ("pos", C.c_int32), ("has_gauss", C.c_int32), ("gauss", C.c_double)]


_VIEW = None
_TRIED = False


def view():
    """The view of numpy's global RandomState, or None when its layout is not the
    one proven above (the caller then uses np.random.get_state / set_state)."""
    global _VIEW, _TRIED
    if _VIEW is not None and not _VIEW.alive():
        _VIEW, _TRIED = None, False
    if not _TRIED:
        _TRIED = True
        try:
            _VIEW = LegacyStateView()
        except Exception:
            _VIEW = None
    return _VIEW
