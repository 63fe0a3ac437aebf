"""Minimal offline reader for binary USD ("USDC crate") files.

Repo tooling, not product code: it runs in the build container only, to turn the reference's
robot asset (``zbot_assets/zbot_6s_new.usd``, crate 0.8.0) into the committed model fixture
``zbot_lab_amd/assets/zbot6s_model.json``. ``pxr`` is not installed, so the crate layout is
decoded here from the published format:

* bootstrap ``PXR-USDC`` + version + TOC offset; TOC of named sections;
* TfFastCompression buffers of LZ4 blocks;
* Usd integer compression (common value + 2-bit width codes + deltas, running sum);
* TOKENS / STRINGS / FIELDS / FIELDSETS / PATHS / SPECS sections;
* 64-bit ValueReps (array / inlined / compressed flags, type id, payload).

Only the value types the ZBOT assets use are decoded; anything else is returned as ``None``.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np


# --------------------------------------------------------------------------- compression
def lz4_block_decompress(src: bytes, out_size_hint: int = 0) -> bytes:
    """Standard LZ4 block format: token (lit_len:4 | match_len:4), literals, 2-byte offset."""
    dst = bytearray()
    i, n = 0, len(src)
    while i < n:
        token = src[i]
        i += 1
        lit = token >> 4
        if lit == 15:
            while True:
                b = src[i]
                i += 1
                lit += b
                if b != 255:
                    break
        dst += src[i:i + lit]
        i += lit
        if i >= n:  # last sequence carries literals only
            break
        off = src[i] | (src[i + 1] << 8)
        i += 2
        mlen = token & 15
        if mlen == 15:
            while True:
                b = src[i]
                i += 1
                mlen += b
                if b != 255:
                    break
        mlen += 4
        start = len(dst) - off
        if off >= mlen:
            dst += dst[start:start + mlen]
        else:  # overlapping copy
            for k in range(mlen):
                dst.append(dst[start + k])
    return bytes(dst)


def tf_fast_decompress(buf: bytes) -> bytes:
    """TfFastCompression: byte 0 = chunk count; 0 => one LZ4 block follows."""
    nchunks = buf[0]
    if nchunks == 0:
        return lz4_block_decompress(buf[1:])
    out, pos = bytearray(), 1
    for _ in range(nchunks):
        (sz,) = struct.unpack_from("<i", buf, pos)
        pos += 4
        out += lz4_block_decompress(buf[pos:pos + sz])
        pos += sz
    return bytes(out)


def decode_ints(enc: bytes, n: int, width: int = 32) -> np.ndarray:
    """Usd integer (de)compression: common value, 2-bit codes (0 common, 1 i8, 2 i16, 3 i32/i64)."""
    big = width == 64
    cfmt, csz = ("<q", 8) if big else ("<i", 4)
    (common,) = struct.unpack_from(cfmt, enc, 0)
    codes_off = csz
    ncode_bytes = (2 * n + 7) // 8
    vpos = codes_off + ncode_bytes
    out = np.empty(n, dtype=np.int64)
    acc = 0
    wide_fmt, wide_sz = (("<q", 8) if big else ("<i", 4))
    for k in range(n):
        code = (enc[codes_off + (k >> 2)] >> (2 * (k & 3))) & 3
        if code == 0:
            d = common
        elif code == 1:
            (d,) = struct.unpack_from("<b", enc, vpos)
            vpos += 1
        elif code == 2:
            (d,) = struct.unpack_from("<h", enc, vpos)
            vpos += 2
        else:
            (d,) = struct.unpack_from(wide_fmt, enc, vpos)
            vpos += wide_sz
        acc += d
        out[k] = acc
    return out


# --------------------------------------------------------------------------- value types
TYPE_NAMES = {
    1: "bool", 2: "uchar", 3: "int", 4: "uint", 5: "int64", 6: "uint64", 7: "half", 8: "float",
    9: "double", 10: "string", 11: "token", 12: "asset", 13: "matrix2d", 14: "matrix3d",
    15: "matrix4d", 16: "quatd", 17: "quatf", 18: "quath", 19: "vec2d", 20: "vec2f", 21: "vec2h",
    22: "vec2i", 23: "vec3d", 24: "vec3f", 25: "vec3h", 26: "vec3i", 27: "vec4d", 28: "vec4f",
    29: "vec4h", 30: "vec4i", 31: "dictionary", 32: "tokenlistop", 33: "stringlistop",
    34: "pathlistop", 35: "referencelistop", 36: "intlistop", 40: "pathvector",
    41: "tokenvector", 42: "specifier", 43: "permission", 44: "variability", 48: "doublevector",
}

# element layout (struct fmt, count) for fixed-size scalar/vector types
_ELEM = {
    "bool": ("<?", 1), "uchar": ("<B", 1), "int": ("<i", 1), "uint": ("<I", 1),
    "int64": ("<q", 1), "uint64": ("<Q", 1), "half": ("<e", 1), "float": ("<f", 1),
    "double": ("<d", 1), "quatd": ("<4d", 4), "quatf": ("<4f", 4), "quath": ("<4e", 4),
    "vec2d": ("<2d", 2), "vec2f": ("<2f", 2), "vec2i": ("<2i", 2), "vec3d": ("<3d", 3),
    "vec3f": ("<3f", 3), "vec3h": ("<3e", 3), "vec3i": ("<3i", 3), "vec4d": ("<4d", 4),
    "vec4f": ("<4f", 4), "vec4i": ("<4i", 4), "matrix4d": ("<16d", 16), "matrix3d": ("<9d", 9),
}


@dataclass
class Spec:
    path: str
    spec_type: int
    fields: dict = field(default_factory=dict)


class Crate:
    def __init__(self, path: str):
        self.data = open(path, "rb").read()
        d = self.data
        if d[:8] != b"PXR-USDC":
            raise ValueError("not a USDC crate")
        self.version = tuple(d[8:11])
        (toc,) = struct.unpack_from("<q", d, 16)
        (nsec,) = struct.unpack_from("<Q", d, toc)
        self.sections = {}
        for s in range(nsec):
            o = toc + 8 + 32 * s
            name = d[o:o + 16].rstrip(b"\0").decode()
            start, size = struct.unpack_from("<qq", d, o + 16)
            self.sections[name] = (start, size)
        self._read_tokens()
        self._read_strings()
        self._read_fields()
        self._read_fieldsets()
        self._read_paths()
        self._read_specs()

    # ---- section readers
    def _compressed_ints(self, pos: int, n: int, width: int = 32):
        (csize,) = struct.unpack_from("<Q", self.data, pos)
        pos += 8
        raw = tf_fast_decompress(self.data[pos:pos + csize])
        return decode_ints(raw, n, width), pos + csize

    def _read_tokens(self):
        start, _ = self.sections["TOKENS"]
        n, usz, csz = struct.unpack_from("<QQQ", self.data, start)
        raw = tf_fast_decompress(self.data[start + 24:start + 24 + csz])
        assert len(raw) == usz, (len(raw), usz)
        toks = raw.split(b"\0")[:n]
        self.tokens = [t.decode("utf-8") for t in toks]

    def _read_strings(self):
        start, _ = self.sections["STRINGS"]
        (n,) = struct.unpack_from("<Q", self.data, start)
        self.strings = list(struct.unpack_from(f"<{n}I", self.data, start + 8))

    def _read_fields(self):
        start, _ = self.sections["FIELDS"]
        (n,) = struct.unpack_from("<Q", self.data, start)
        toks, pos = self._compressed_ints(start + 8, n)
        (rsz,) = struct.unpack_from("<Q", self.data, pos)
        reps = tf_fast_decompress(self.data[pos + 8:pos + 8 + rsz])
        reps = struct.unpack(f"<{n}Q", reps[:8 * n])
        self.fields = [(self.tokens[int(t)], r) for t, r in zip(toks, reps)]

    def _read_fieldsets(self):
        start, _ = self.sections["FIELDSETS"]
        (n,) = struct.unpack_from("<Q", self.data, start)
        vals, _ = self._compressed_ints(start + 8, n)
        self.fieldsets = [int(v) & 0xFFFFFFFF for v in vals]

    def _read_paths(self):
        start, _ = self.sections["PATHS"]
        npaths, nenc = struct.unpack_from("<QQ", self.data, start)
        pos = start + 16
        pidx, pos = self._compressed_ints(pos, nenc)
        etok, pos = self._compressed_ints(pos, nenc)
        jumps, pos = self._compressed_ints(pos, nenc)
        self.paths = [None] * npaths
        self._build_paths(pidx, etok, jumps, 0, None)

    def _build_paths(self, pidx, etok, jumps, cur, parent):
        while True:
            i = cur
            cur += 1
            if parent is None:
                parent = "/"
                self.paths[pidx[i]] = parent
            else:
                t = int(etok[i])
                is_prop = t < 0
                name = self.tokens[abs(t)]
                if is_prop:
                    p = parent + "." + name
                elif parent == "/":
                    p = "/" + name
                else:
                    p = parent + "/" + name
                self.paths[pidx[i]] = p
            has_child = jumps[i] > 0 or jumps[i] == -1
            has_sib = jumps[i] >= 0
            if has_child:
                if has_sib:
                    self._build_paths(pidx, etok, jumps, i + int(jumps[i]), parent)
                parent = self.paths[pidx[i]]
            elif not has_sib:
                break

    def _read_specs(self):
        start, _ = self.sections["SPECS"]
        (n,) = struct.unpack_from("<Q", self.data, start)
        pos = start + 8
        pidx, pos = self._compressed_ints(pos, n)
        fsidx, pos = self._compressed_ints(pos, n)
        stype, pos = self._compressed_ints(pos, n)
        self.specs = {}
        for p, f, t in zip(pidx, fsidx, stype):
            fl = {}
            k = int(f)
            while self.fieldsets[k] != 0xFFFFFFFF:
                name, rep = self.fields[self.fieldsets[k]]
                fl[name] = rep
                k += 1
            path = self.paths[int(p)]
            self.specs[path] = Spec(path, int(t), fl)

    # ---- value decoding
    def value(self, rep: int):
        is_array = bool(rep >> 63 & 1)
        inlined = bool(rep >> 62 & 1)
        compressed = bool(rep >> 61 & 1)
        tid = (rep >> 48) & 0xFF
        payload = rep & ((1 << 48) - 1)
        tname = TYPE_NAMES.get(tid)
        d = self.data
        if tname is None:
            return None
        if inlined:
            pb = struct.pack("<Q", payload)
            if tname in ("token",):
                return self.tokens[payload]
            if tname == "string":
                return self.tokens[self.strings[payload]]
            if tname in ("float", "double"):
                return struct.unpack("<f", pb[:4])[0]
            if tname in ("int", "uint", "bool", "uchar", "specifier", "variability", "permission"):
                return struct.unpack("<i", pb[:4])[0]
            if tname.startswith("vec") or tname.startswith("quat"):
                nc = int(tname[3]) if tname.startswith("vec") else 4
                return tuple(struct.unpack(f"<{nc}b", pb[:nc]))
            if tname == "matrix4d":  # inlined diagonal
                diag = struct.unpack("<4b", pb[:4])
                return np.diag(np.array(diag, dtype=np.float64))
            return payload
        pos = payload
        if tname == "tokenvector":
            (n,) = struct.unpack_from("<Q", d, pos)
            idx = struct.unpack_from(f"<{n}I", d, pos + 8)
            return [self.tokens[i] for i in idx]
        if tname == "pathlistop":
            return self._pathlistop(pos)
        if tname == "tokenlistop":
            return self._tokenlistop(pos)
        if tname == "dictionary":
            return None
        if tname == "token" and is_array:
            (n,) = struct.unpack_from("<Q", d, pos)
            idx = struct.unpack_from(f"<{n}I", d, pos + 8)
            return [self.tokens[i] for i in idx]
        if tname in _ELEM:
            fmt, nc = _ELEM[tname]
            esz = struct.calcsize(fmt)
            if is_array:
                (n,) = struct.unpack_from("<Q", d, pos)
                pos += 8
                if compressed:
                    if tname in ("int", "uint"):
                        vals, _ = self._compressed_ints(pos, n)
                        return vals
                    return None  # compressed float arrays not needed here
                arr = np.frombuffer(d, dtype=np.dtype(fmt[1:] if nc == 1 else fmt[-1]).newbyteorder("<"),
                                    count=n * nc, offset=pos)
                return arr.reshape(n, nc) if nc > 1 else arr
            v = struct.unpack_from(fmt, d, pos)
            return v if nc > 1 else v[0]
        return None

    def _paths_list(self, pos):
        (n,) = struct.unpack_from("<Q", self.data, pos)
        idx = struct.unpack_from(f"<{n}I", self.data, pos + 8)
        return [self.paths[i] for i in idx], pos + 8 + 4 * n

    def _pathlistop(self, pos):
        hdr = self.data[pos]
        pos += 1
        out = {}
        for bit, name in ((1, "explicit_flag"), (2, "explicit"), (4, "added"), (8, "deleted"),
                          (16, "ordered"), (32, "prepended"), (64, "appended")):
            if bit == 1:
                continue
            if hdr & bit:
                out[name], pos = self._paths_list(pos)
        return out

    def _tokenlistop(self, pos):
        hdr = self.data[pos]
        pos += 1
        out = {}
        for bit, name in ((2, "explicit"), (4, "added"), (8, "deleted"), (16, "ordered"),
                          (32, "prepended"), (64, "appended")):
            if hdr & bit:
                (n,) = struct.unpack_from("<Q", self.data, pos)
                idx = struct.unpack_from(f"<{n}I", self.data, pos + 8)
                out[name] = [self.tokens[i] for i in idx]
                pos += 8 + 4 * n
        return out

    # ---- convenience
    def get(self, path: str, fname: str = "default"):
        s = self.specs.get(path)
        if s is None or fname not in s.fields:
            return None
        return self.value(s.fields[fname])

    def children(self, prim: str):
        pre = prim.rstrip("/") + "/"
        out = []
        for p in self.specs:
            if p.startswith(pre) and "." not in p[len(pre):] and "/" not in p[len(pre):]:
                out.append(p)
        return out
