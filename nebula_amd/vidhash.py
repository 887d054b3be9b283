"""VID helpers for fixtures.

The reference test fixtures derive vertex ids as ``std::hash<std::string>()(name)``
(``src/graph/test/TraverseTestBase.h:111,233``) and nGQL's ``hash()`` builtin uses the
same function (``src/common/filter/FunctionManager.cpp``).  With libstdc++ that is
``std::_Hash_bytes(data, len, 0xc70f6907)`` — the 64-bit MurmurHash2 variant below —
reinterpreted as a signed int64 VertexID.
"""

_M = 0xC6A4A7935BD1E995
_MASK = (1 << 64) - 1


def _shift_mix(v: int) -> int:
    return v ^ (v >> 47)


def std_hash(s: str | bytes, seed: int = 0xC70F6907) -> int:
    """libstdc++ ``std::_Hash_bytes`` for 64-bit size_t, returned as signed int64."""
    data = s.encode() if isinstance(s, str) else s
    n = len(data)
    aligned = n & ~7
    h = (seed ^ ((n * _M) & _MASK)) & _MASK
    for i in range(0, aligned, 8):
        k = int.from_bytes(data[i:i + 8], "little")
        data_ = (_shift_mix((k * _M) & _MASK) * _M) & _MASK
        h ^= data_
        h = (h * _M) & _MASK
    tail = n & 7
    if tail:
        # load_bytes: little-endian accumulation of the trailing bytes
        v = 0
        for j in range(tail - 1, -1, -1):
            v = (v << 8) + data[aligned + j]
        h ^= v
        h = (h * _M) & _MASK
    h = (_shift_mix(h) * _M) & _MASK
    h = _shift_mix(h)
    return h - (1 << 64) if h >= (1 << 63) else h
