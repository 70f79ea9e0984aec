"""Resource requirements: ranges, memory sizes, the GPU spec grammar (reference:
``C/models/resources.py:19-292``).

The GPU grammar is ``[vendor:][name[,name...]][:memory][:count]`` in any order, e.g. ``MI355X:8``,
``amd:288GB:8``, ``MI300X,MI355X:4..8``, ``24GB..:2``. AMD Instinct names are first-class:
``vendor`` is inferred as ``amd`` for ``MI*`` names when not given.
"""

from __future__ import annotations

import math
from enum import Enum
from typing import Any, Generic, List, Optional, Tuple, TypeVar, Union

from pydantic import Field, GetCoreSchemaHandler, field_validator, model_validator
from pydantic_core import core_schema

from dstack_amd.core.models.common import CoreModel

T = TypeVar("T", int, float)


class Memory(float):
    """Memory size in GB. Accepts numbers and ``"512MB"``, ``"80GB"``, ``"1.5TB"``."""

    @classmethod
    def parse(cls, v: Any) -> "Memory":
        if isinstance(v, bool):
            raise ValueError(f"Invalid memory size: {v}")
        if isinstance(v, (int, float)):
            return cls(v)
        if isinstance(v, str):
            s = v.replace(" ", "").lower()
            try:
                if s.endswith("tb"):
                    return cls(float(s[:-2]) * 1024)
                if s.endswith("gb"):
                    return cls(float(s[:-2]))
                if s.endswith("mb"):
                    return cls(float(s[:-2]) / 1024)
                return cls(float(s))
            except ValueError:
                pass
        raise ValueError(f"Invalid memory size: {v!r}")

    def __repr__(self) -> str:
        return f"{self:g}GB"

    def __str__(self) -> str:
        return f"{self:g}GB"

    @classmethod
    def __get_pydantic_core_schema__(cls, source, handler: GetCoreSchemaHandler):
        return core_schema.no_info_plain_validator_function(
            cls.parse,
            json_schema_input_schema=core_schema.union_schema([core_schema.float_schema(), core_schema.str_schema()]),
            serialization=core_schema.plain_serializer_function_ser_schema(float, return_schema=core_schema.float_schema()),
        )


class Range(CoreModel, Generic[T]):
    """Closed range ``min..max`` with either end open. Parses ``"2"``, ``"2.."``, ``"..8"``,
    ``"2..8"`` and numbers."""

    min: Optional[T] = None
    max: Optional[T] = None

    @model_validator(mode="before")
    @classmethod
    def _parse(cls, v: Any) -> Any:
        if isinstance(v, Range):
            return {"min": v.min, "max": v.max}
        if isinstance(v, str):
            s = v.replace(" ", "")
            if ".." in s:
                lo, hi = s.split("..", 1)
                return {"min": lo or None, "max": hi or None}
            return {"min": s, "max": s}
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            return {"min": v, "max": v}
        return v

    @model_validator(mode="after")
    def _check(self):
        if self.min is None and self.max is None:
            raise ValueError("Invalid empty range: ..")
        if self.min is not None and self.max is not None and self.min > self.max:
            raise ValueError(f"Invalid range order: {self.min}..{self.max}")
        return self

    def __str__(self) -> str:
        lo = "" if self.min is None else _fmt(self.min)
        hi = "" if self.max is None else _fmt(self.max)
        return lo if lo == hi else f"{lo}..{hi}"

    def contains(self, x: float) -> bool:
        return (self.min is None or x >= self.min) and (self.max is None or x <= self.max)

    def intersect(self, other: "Range") -> Optional["Range"]:
        start = max(self.min if self.min is not None else -math.inf, other.min if other.min is not None else -math.inf)
        end = min(self.max if self.max is not None else math.inf, other.max if other.max is not None else math.inf)
        if start > end:
            return None
        return type(self)(min=None if math.isinf(start) else start, max=None if math.isinf(end) else end)


def _fmt(x) -> str:
    if isinstance(x, Memory):
        return str(x)
    if isinstance(x, float) and x.is_integer():
        return str(int(x))
    return str(x)


class IntRange(Range[int]):
    pass


class MemoryRange(Range[Memory]):
    pass


class AcceleratorVendor(str, Enum):
    NVIDIA = "nvidia"
    AMD = "amd"
    GOOGLE = "google"
    INTEL = "intel"

    @classmethod
    def cast(cls, v: str) -> "AcceleratorVendor":
        v = v.lower()
        if v == "tpu":
            return cls.GOOGLE
        return cls(v)


class ComputeCapability(tuple):
    @classmethod
    def parse(cls, v: Any) -> Tuple[int, int]:
        if isinstance(v, float):
            v = str(v)
        if isinstance(v, str):
            v = v.strip().split(".")
        if isinstance(v, (tuple, list)) and len(v) == 2:
            return cls((int(v[0]), int(v[1])))
        raise ValueError(f"Invalid compute capability: {v}")

    @classmethod
    def __get_pydantic_core_schema__(cls, source, handler: GetCoreSchemaHandler):
        return core_schema.no_info_plain_validator_function(
            cls.parse, json_schema_input_schema=core_schema.str_schema(),
            serialization=core_schema.plain_serializer_function_ser_schema(lambda x: f"{x[0]}.{x[1]}",
                                                                            return_schema=core_schema.str_schema()),
        )


DEFAULT_CPU_COUNT = IntRange(min=2)
DEFAULT_MEMORY_SIZE = MemoryRange(min=Memory(8))
DEFAULT_GPU_COUNT = IntRange(min=1, max=1)


def _vendor_or_none(token: str) -> Optional[AcceleratorVendor]:
    try:
        return AcceleratorVendor.cast(token)
    except ValueError:
        return None


class GPUSpec(CoreModel):
    vendor: Optional[AcceleratorVendor] = Field(None, description="nvidia, amd, google (tpu), intel")
    name: Optional[List[str]] = Field(None, description="GPU names, e.g. MI355X")
    count: IntRange = Field(default_factory=lambda: IntRange(min=1, max=1))
    memory: Optional[MemoryRange] = Field(None, description="Per-GPU memory, e.g. 192GB..")
    total_memory: Optional[MemoryRange] = None
    compute_capability: Optional[ComputeCapability] = None

    @model_validator(mode="before")
    @classmethod
    def _parse(cls, v: Any) -> Any:
        if isinstance(v, bool):
            raise ValueError(f"Invalid GPU spec: {v}")
        if isinstance(v, int):
            v = str(v)
        if isinstance(v, str):
            spec: dict = {}
            for token in v.replace(" ", "").split(":"):
                if not token:
                    raise ValueError(f"GPU spec contains empty token: {v}")
                vendor = _vendor_or_none(token)
                if vendor is not None:
                    if "vendor" in spec:
                        raise ValueError(f"GPU spec vendor conflict: {v}")
                    spec["vendor"] = vendor
                elif token[0].isalpha():
                    if "name" in spec:
                        raise ValueError(f"GPU spec name conflict: {v}")
                    spec["name"] = token.split(",")
                    if any(not n for n in spec["name"]):
                        raise ValueError(f"GPU name can not be empty: {v}")
                elif any(c.isalpha() for c in token):
                    if "memory" in spec:
                        raise ValueError(f"GPU spec memory conflict: {v}")
                    spec["memory"] = token
                else:
                    if "count" in spec:
                        raise ValueError(f"GPU spec count conflict: {v}")
                    spec["count"] = token
            return spec
        return v

    @field_validator("name", mode="before")
    @classmethod
    def _names(cls, v):
        if v is None:
            return None
        if not isinstance(v, list):
            v = [v]
        return [n[4:] if isinstance(n, str) and n.startswith("tpu-") else n for n in v]

    @field_validator("vendor", mode="before")
    @classmethod
    def _vendor(cls, v):
        if isinstance(v, str):
            return AcceleratorVendor.cast(v)
        return v

    @model_validator(mode="after")
    def _infer_vendor(self):
        if self.vendor is None and self.name:
            from dstack_amd.core.models.gpus import vendor_of

            vendors = {vendor_of(n) for n in self.name}
            if len(vendors) == 1 and None not in vendors:
                self.vendor = vendors.pop()
        return self

    def __str__(self) -> str:
        parts = []
        if self.name:
            parts.append(",".join(self.name))
        if self.memory:
            parts.append(str(self.memory))
        parts.append(str(self.count))
        return ":".join(parts)


class DiskSpec(CoreModel):
    size: MemoryRange

    @model_validator(mode="before")
    @classmethod
    def _parse(cls, v: Any) -> Any:
        if isinstance(v, (str, int, float)) and not isinstance(v, bool):
            return {"size": v}
        return v


DEFAULT_DISK = DiskSpec(size=MemoryRange(min=Memory(100)))


class CPUSpec(IntRange):
    pass


class ResourcesSpec(CoreModel):
    cpu: IntRange = Field(default_factory=lambda: IntRange(min=2))
    memory: MemoryRange = Field(default_factory=lambda: MemoryRange(min=Memory(8)))
    shm_size: Optional[Memory] = None
    gpu: Optional[GPUSpec] = None
    disk: Optional[DiskSpec] = Field(default_factory=lambda: DiskSpec(size=MemoryRange(min=Memory(100))))

    def pretty_format(self) -> str:
        parts = [f"{self.cpu}xCPU", f"{self.memory}"]
        if self.gpu:
            g = self.gpu
            s = f"{g.count}x" + (",".join(g.name) if g.name else "GPU")
            if g.memory:
                s += f" ({g.memory})"
            parts.append(s)
        if self.disk:
            parts.append(f"{self.disk.size} (disk)")
        return ", ".join(parts)


ResourcesSpecLike = Union[ResourcesSpec, dict]
