"""Mirror of knossos.model for this path.

The demo checks (model/cas-register) (etcdemo.clj:117).
(model/register) and (model/mutex) are the other Knossos models whose state
space maps onto the device's transition descriptors (include/lincheck.h
LC_T_*, LC_MODEL_*); (model/multi-register) runs on the
set tiers through a per-key transition table (lc_batch.table).  The step functions here only
produce the result maps' :model values and "can't ..." messages on the host;
the search itself runs on the device.  Messages follow the public knossos
0.3.7 source as recalled (not verifiable here: knossos is absent).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from . import _native as N


@dataclass(frozen=True)
class Inconsistent:
    msg: str


def fmt(v) -> str:
    return "nil" if v is None else str(v)


@dataclass(frozen=True)
class CASRegister:
    """knossos.model/cas-register: nil initial value unless given."""
    value: Optional[int] = None
    code = N.LC_MODEL_CAS_REGISTER
    name = "cas-register"

    def step(self, f: str, v):
        if f == "write":
            return CASRegister(v)
        if f == "cas":
            cur, new = v
            if cur == self.value:
                return CASRegister(new)
            return Inconsistent(f"can't CAS {fmt(self.value)} from {fmt(cur)} to {fmt(new)}")
        if f == "read":
            if v is None or v == self.value:
                return self
            return Inconsistent(f"can't read {fmt(v)} from register {fmt(self.value)}")
        raise ValueError(f"cas-register cannot step {f!r}")

    def of_state(self, value):
        return CASRegister(value)

    def render(self) -> dict:
        return {"value": self.value}


@dataclass(frozen=True)
class Register:
    """knossos.model/register: read / write, nil initial value."""
    value: Optional[int] = None
    code = N.LC_MODEL_REGISTER
    name = "register"

    def step(self, f: str, v):
        if f == "write":
            return Register(v)
        if f == "read":
            if v is None or v == self.value:
                return self
            return Inconsistent(f"{fmt(self.value)}≠{fmt(v)}")
        raise ValueError(f"register cannot step {f!r}")

    def of_state(self, value):
        return Register(value)

    def render(self) -> dict:
        return {"value": self.value}


@dataclass(frozen=True)
class Mutex:
    """knossos.model/mutex: unlocked initially."""
    locked: bool = False
    code = N.LC_MODEL_MUTEX
    name = "mutex"

    def step(self, f: str, v=None):
        if f == "acquire":
            return Inconsistent("already held") if self.locked else Mutex(True)
        if f == "release":
            return Mutex(False) if self.locked else Inconsistent("not held")
        raise ValueError(f"mutex cannot step {f!r}")

    def of_state(self, value):
        # lc_pack numbers the mutex states 0 = unlocked (nil), 1 = locked
        return Mutex(value is not None)

    def render(self) -> dict:
        return {"locked?": self.locked}


@dataclass(frozen=True)
class MultiRegister:
    """knossos.model/multi-register: a map of registers; one :f, :txn, whose
    value is a sequence of [:read k v] / [:write k v] micro-ops applied in
    order.  A read of v is legal iff v is nil or register k holds v."""
    registers: tuple = ()   # ((register, value), ...) in register order
    code = N.LC_MODEL_MULTI_REGISTER
    name = "multi-register"

    @staticmethod
    def _order(kv):
        return (str(type(kv[0])), kv[0])

    def step(self, f: str, v):
        if f != "txn":
            raise ValueError(f"multi-register cannot step {f!r}")
        regs = dict(self.registers)
        for mf, k, x in (v or ()):
            mf = str(mf).lstrip(":")
            if mf == "read":
                if x is not None and (k not in regs or regs[k] != x):
                    return Inconsistent(f"{fmt(regs.get(k))}≠{fmt(x)}")
            elif mf == "write":
                regs[k] = x
            else:
                raise ValueError(f"multi-register cannot step micro-op {mf!r}")
        return MultiRegister(tuple(sorted(regs.items(), key=self._order)))

    def init_pairs(self, reg_id) -> list:
        """(register id, value) pairs of the initial map for lc_pack_opts."""
        return [(reg_id(k), v) for k, v in self.registers]

    def of_map(self, pairs):
        return MultiRegister(tuple(sorted(pairs, key=self._order)))

    def render(self) -> dict:
        return dict(self.registers)


def cas_register(value: Optional[int] = None) -> CASRegister:
    if value is not None:
        raise NotImplementedError("only the nil initial value of (model/cas-register) is supported")
    return CASRegister(value)


def register(value: Optional[int] = None) -> Register:
    if value is not None:
        raise NotImplementedError("only the nil initial value of (model/register) is supported")
    return Register(value)


def mutex() -> Mutex:
    return Mutex(False)


def multi_register(values: Optional[dict] = None) -> MultiRegister:
    """(model/multi-register values): values maps registers to initial values."""
    return MultiRegister(tuple(sorted((values or {}).items(), key=MultiRegister._order)))


MODELS = (CASRegister, Register, Mutex, MultiRegister)
