"""Lockset race detector for the Python side of the runtime.

The reference has no concurrency control at all: FastAPI runs concurrent /generate
calls in anyio's threadpool over shared module globals (`server.py:154-155`).  Here
the Python runtime is multi-threaded by design -- the serving loop, HTTP handler
threads submitting requests, in-process stage threads (local / loopback pipelines),
DP token receivers and the progress watchdog -- and its shared mutable state is
meant to be guarded by locks.  The native parts (request queue, scheduler core) are
covered by TSan / ASan stress drivers (csrc/runtime/tests); CPython cannot run under
TSan, so this module checks the Python side with the Eraser lockset algorithm
(Savage et al., SOSP'97), restricted to writes:

  * locks made through `Lock()` / `RLock()` / `Condition()` here record, per thread,
    which of them the thread holds;
  * every attribute write on a `Shared` object, and every `note(obj, field)` call at
    a container mutation, updates that field's state: Exclusive(first writer thread)
    until a second thread writes it, then Shared with candidate lockset C = the locks
    held at that write, intersected with the locks held at every later write;
  * a field whose candidate lockset becomes empty is reported: two threads write it
    with no lock in common.

`handoff(obj)` resets an object's fields (ownership moves to another thread at a
synchronisation point the detector cannot see, e.g. a thread start/join).

Enabled by LSD_RACE_CHECK=1 in the environment before import; otherwise `Lock` &c.
return the plain `threading` primitives and `Shared` is `object`: zero cost.
"""
from __future__ import annotations

import collections
import os
import threading
import traceback
import weakref
from typing import Dict, List, Optional, Tuple

ENABLED = os.environ.get("LSD_RACE_CHECK", "0") == "1"

_tls = threading.local()
_state_lock = threading.Lock()
# (id(obj), field) -> [owner thread ident or None (shared), lockset (frozenset) or None, reported]
_state: Dict[Tuple[int, str], list] = {}
_final: set = set()  # ids with a finalizer registered
_reports: List[dict] = []
# ids of dead objects whose write history is still to be dropped: a finalizer
# may run inside ANY allocation -- also one made while this thread holds
# _state_lock (the weakref.finalize call in note() allocates, a collection
# it triggers finalizes some other object) -- so finalizers only queue the id
# (deque.append: atomic, takes no lock) and the next locked section drops it,
# before it can look up a key of an object that reused the id
_dead: "collections.deque[int]" = collections.deque()


def _held() -> list:
    h = getattr(_tls, "held", None)
    if h is None:
        h = _tls.held = []
    return h


class _TrackedLock:
    """threading.Lock / RLock wrapper that records the locks each thread holds."""

    def __init__(self, inner, name: Optional[str]):
        self._inner = inner
        self.name = name or f"lock@{id(self):x}"

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        ok = self._inner.acquire(blocking, timeout)
        if ok:
            _held().append(self)
        return ok

    def release(self) -> None:
        h = _held()
        for i in range(len(h) - 1, -1, -1):
            if h[i] is self:
                del h[i]
                break
        self._inner.release()

    __enter__ = acquire

    def __exit__(self, *exc) -> None:
        self.release()

    # threading.Condition protocol for a re-entrant lock (wait() releases every level)
    def _is_owned(self) -> bool:
        if hasattr(self._inner, "_is_owned"):
            return self._inner._is_owned()
        return any(x is self for x in _held())

    def _release_save(self):
        h = _held()
        n = sum(1 for x in h if x is self)
        h[:] = [x for x in h if x is not self]
        st = self._inner._release_save() if hasattr(self._inner, "_release_save") else self._inner.release()
        return st, n

    def _acquire_restore(self, saved) -> None:
        st, n = saved
        if hasattr(self._inner, "_acquire_restore"):
            self._inner._acquire_restore(st)
        else:
            self._inner.acquire()
        _held().extend([self] * n)

    def locked(self) -> bool:
        return self._inner.locked() if hasattr(self._inner, "locked") else self._is_owned()


def Lock(name: Optional[str] = None):
    return _TrackedLock(threading.Lock(), name) if ENABLED else threading.Lock()


def RLock(name: Optional[str] = None):
    return _TrackedLock(threading.RLock(), name) if ENABLED else threading.RLock()


def Condition(lock=None, name: Optional[str] = None):
    if not ENABLED:
        return threading.Condition(lock)
    return threading.Condition(lock if lock is not None else RLock(name))


def note(obj, field: str) -> None:
    """One write of `field` of `obj` by the calling thread (container mutations)."""
    if not ENABLED:
        return
    me = threading.get_ident()
    held = frozenset(id(x) for x in _held())
    key = (id(obj), field)
    with _state_lock:
        _drop_dead()
        st = _state.get(key)
        if st is None:
            _state[key] = [me, None, False]
            if key[0] not in _final:
                try:  # forget the object's fields when it dies (ids are reused)
                    weakref.finalize(obj, _forget, key[0])
                    _final.add(key[0])
                except TypeError:
                    pass
            return
        owner, lockset, reported = st
        if owner == me and lockset is None:
            return  # still exclusive to its first writer
        lockset = held if lockset is None else (lockset & held)
        st[0], st[1] = None, lockset
        if not lockset and not reported:
            st[2] = True
            names = [x.name for x in _held()]
            _reports.append({"object": type(obj).__name__, "field": field,
                             "thread": threading.current_thread().name, "held": names,
                             "stack": "".join(traceback.format_stack(limit=8)[:-1])})


def _forget(oid: int) -> None:
    _dead.append(oid)


def _drop_dead() -> None:
    """Under _state_lock: drop the write history of the objects that died."""
    while _dead:
        oid = _dead.popleft()
        _final.discard(oid)
        for k in [k for k in _state if k[0] == oid]:
            del _state[k]


def handoff(obj) -> None:
    """Forget the write history of `obj`: its next writer becomes its exclusive owner."""
    if not ENABLED:
        return
    oid = id(obj)
    with _state_lock:
        _drop_dead()
        for k in [k for k in _state if k[0] == oid]:
            del _state[k]


def reports() -> List[dict]:
    with _state_lock:
        return list(_reports)


def reset() -> None:
    with _state_lock:
        _dead.clear()
        _state.clear()
        _final.clear()
        _reports.clear()


if ENABLED:
    class Shared:
        """Mixin: attribute writes are checked (fields starting with '_rc' are not)."""

        def __setattr__(self, name, value):
            object.__setattr__(self, name, value)
            if not name.startswith("_rc"):
                note(self, name)
else:
    Shared = object
