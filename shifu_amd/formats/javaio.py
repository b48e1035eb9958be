"""Java ``DataInput`` / ``DataOutput`` (big-endian) including modified-UTF-8 ``writeUTF``."""
from __future__ import annotations

import gzip
import io
import struct


class JavaOut:
    def __init__(self):
        self.b = io.BytesIO()

    def int(self, v):
        self.b.write(struct.pack(">i", int(v)))

    def long(self, v):
        self.b.write(struct.pack(">q", int(v)))

    def short(self, v):
        self.b.write(struct.pack(">h", int(v)))

    def byte(self, v):
        self.b.write(struct.pack(">b", int(v) if int(v) < 128 else int(v) - 256))

    def bool(self, v):
        self.b.write(b"\x01" if v else b"\x00")

    def float(self, v):
        self.b.write(struct.pack(">f", float(v)))

    def double(self, v):
        self.b.write(struct.pack(">d", float(v)))

    def raw(self, bs: bytes):
        self.b.write(bs)

    def utf(self, s: str):
        """DataOutput.writeUTF: 2-byte length + modified UTF-8 (NUL as C0 80, supplementary as surrogates)."""
        enc = bytearray()
        for ch in s:
            c = ord(ch)
            if c > 0xFFFF:
                c -= 0x10000
                for u in (0xD800 + (c >> 10), 0xDC00 + (c & 0x3FF)):
                    enc += bytes([0xE0 | (u >> 12), 0x80 | ((u >> 6) & 0x3F), 0x80 | (u & 0x3F)])
            elif 0 < c < 0x80:
                enc.append(c)
            elif c < 0x800:
                enc += bytes([0xC0 | (c >> 6), 0x80 | (c & 0x3F)])
            else:
                enc += bytes([0xE0 | (c >> 12), 0x80 | ((c >> 6) & 0x3F), 0x80 | (c & 0x3F)])
        if len(enc) > 65535:
            raise ValueError("writeUTF string too long")
        self.short(len(enc) if len(enc) < 32768 else len(enc) - 65536)
        self.b.write(bytes(enc))

    def string(self, s: str | None):
        """Shifu ``StringUtils.writeString``: int length + UTF-8 bytes (null -> 0)."""
        if s is None:
            self.int(0)
            return
        bs = s.encode("utf-8")
        self.int(len(bs))
        self.b.write(bs)

    def int_array(self, a):
        if a is None:
            self.int(0)
            return
        self.int(len(a))
        for v in a:
            self.int(v)

    def double_array(self, a):
        if a is None:
            self.int(0)
            return
        self.int(len(a))
        self.b.write(struct.pack(f">{len(a)}d", *[float(x) for x in a]))

    def bytes(self) -> bytes:
        return self.b.getvalue()

    def gzip_bytes(self) -> bytes:
        return gzip.compress(self.bytes(), mtime=0)


class JavaIn:
    def __init__(self, data: bytes):
        if data[:2] == b"\x1f\x8b":
            data = gzip.decompress(data)
        self.d = data
        self.p = 0

    def _take(self, n):
        if self.p + n > len(self.d):
            raise EOFError("unexpected end of stream")
        v = self.d[self.p: self.p + n]
        self.p += n
        return v

    def int(self):
        return struct.unpack(">i", self._take(4))[0]

    def long(self):
        return struct.unpack(">q", self._take(8))[0]

    def short(self):
        return struct.unpack(">h", self._take(2))[0]

    def ushort(self):
        return struct.unpack(">H", self._take(2))[0]

    def byte(self):
        return struct.unpack(">b", self._take(1))[0]

    def bool(self):
        return self._take(1) != b"\x00"

    def float(self):
        return struct.unpack(">f", self._take(4))[0]

    def double(self):
        return struct.unpack(">d", self._take(8))[0]

    def utf(self) -> str:
        n = self.ushort()
        return decode_modified_utf8(self._take(n))

    def string(self):
        n = self.int()
        if n == 0:
            return None
        return self._take(n).decode("utf-8")

    def int_array(self):
        n = self.int()
        return [self.int() for _ in range(n)]

    def double_array(self):
        n = self.int()
        return list(struct.unpack(f">{n}d", self._take(8 * n))) if n else []

    def eof(self):
        return self.p >= len(self.d)


def decode_modified_utf8(bs: bytes) -> str:
    out, i, n = [], 0, len(bs)
    while i < n:
        c = bs[i]
        if c < 0x80:
            out.append(c); i += 1
        elif c >> 5 == 0x6:
            out.append(((c & 0x1F) << 6) | (bs[i + 1] & 0x3F)); i += 2
        else:
            out.append(((c & 0x0F) << 12) | ((bs[i + 1] & 0x3F) << 6) | (bs[i + 2] & 0x3F)); i += 3
    # merge surrogate pairs
    s = []
    k = 0
    while k < len(out):
        u = out[k]
        if 0xD800 <= u < 0xDC00 and k + 1 < len(out) and 0xDC00 <= out[k + 1] < 0xE000:
            s.append(chr(0x10000 + ((u - 0xD800) << 10) + (out[k + 1] - 0xDC00))); k += 2
        else:
            s.append(chr(u)); k += 1
    return "".join(s)
