"""Reader for oracle/ref_probe's tagged binary records (test tooling only)."""
import struct
import numpy as np

_DT = {b'f': np.float32, b'i': np.int32, b'd': np.float64, b'q': np.int64, b'c': np.uint8, b'h': np.uint16}


def read(path):
    out = {}
    with open(path, 'rb') as fh:
        buf = fh.read()
    off = 0
    while off < len(buf):
        (n,) = struct.unpack_from('<I', buf, off); off += 4
        name = buf[off:off + n].decode(); off += n
        dt = buf[off:off + 1]; off += 1
        (cnt,) = struct.unpack_from('<Q', buf, off); off += 8
        t = np.dtype(_DT[dt])
        out[name] = np.frombuffer(buf, dtype=t, count=cnt, offset=off).copy()
        off += cnt * t.itemsize
    return out
