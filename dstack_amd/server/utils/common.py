"""Byte-stream helpers (reference ``server/utils/common.py:45``)."""

from __future__ import annotations

from typing import AsyncIterable, Iterable, Optional


def join_byte_stream_checked(stream: Iterable[bytes], max_size: int) -> Optional[bytes]:
    """Concatenate ``stream`` unless it holds more than ``max_size`` bytes, in which case return
    None without pulling another chunk once the limit is crossed (a remote body is never read
    past the limit)."""
    buf = bytearray()
    for chunk in stream:
        buf += chunk
        if len(buf) > max_size:
            return None
    return bytes(buf)


async def ajoin_byte_stream_checked(stream: AsyncIterable[bytes], max_size: int) -> Optional[bytes]:
    """``join_byte_stream_checked`` for an async stream (an HTTP request body)."""
    buf = bytearray()
    async for chunk in stream:
        buf += chunk
        if len(buf) > max_size:
            return None
    return bytes(buf)
