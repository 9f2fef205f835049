"""Host-side mirror of the reference's StorageBlock topology (src/vfs/block.rs:22-98).

The VirtualBlock/VirtualFile glue around the codec (sync_data / load_block)
is added on top of ``ReedSolomon`` in later rounds.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Union


@dataclass(frozen=True)
class Single:
    def __str__(self) -> str:
        return "Single"


@dataclass(frozen=True)
class Mirror:
    n: int

    def __str__(self) -> str:
        return f"Mirror({self.n})"


@dataclass(frozen=True)
class Erasure:
    version: int
    data: int
    parity: int

    def __str__(self) -> str:
        return f"Erasure({self.version}, {self.data}, {self.parity})"


BlockTopology = Union[Single, Mirror, Erasure]


def _u8(s: str) -> int:
    v = int(s.strip())
    if not 0 <= v <= 255:
        raise ValueError(s)
    return v


def parse_topology(value: str) -> BlockTopology:
    """``BlockTopology::try_from(String)`` (src/vfs/block.rs:51-98).

    Quirks kept: the text must contain '('; the last character is dropped
    before parsing arguments; "Single" without parentheses fails.
    """
    parts = value.split("(", 1)
    if len(parts) != 2:
        raise ValueError(f"'{value}' does not have '('")
    name, arg = parts[0], parts[1][:-1]
    if name == "Single":
        return Single()
    if name == "Mirror":
        try:
            return Mirror(_u8(arg.rstrip(")")))
        except ValueError:
            raise ValueError(f"Unable to parse {value}. {name} - {arg}") from None
    if name == "Erasure":
        params = arg.split(",", 2)
        try:
            v = _u8(params[0])
        except ValueError:
            raise ValueError(f"Unable to parse version {params}") from None
        try:
            d = _u8(params[1] if len(params) > 1 else "")
        except ValueError:
            raise ValueError(f"Unable to parse data shards {params}") from None
        try:
            p = _u8((params[2] if len(params) > 2 else "").strip().rstrip(")"))
        except ValueError:
            raise ValueError(f"Unable to parse parity shards {params}") from None
        return Erasure(v, d, p)
    raise ValueError(f"Unable to parse {value}. {name} - {arg}")
