"""Register / scratch / LDS use of the gfx950 kernels in a HIP object or shared library, read
on the host (no GPU): the offload bundle in the .hip_fatbin section is split into its code
objects and llvm-readelf --notes prints each kernel's metadata. Used to check a kernel change
for VGPR growth and scratch spills before spending GPU time.
usage: python scripts/kernel_resources.py deepfmkit_amd/dfmi_capi.o [name-substring ...]"""
import os
import re
import struct
import subprocess
import sys
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    data = open(path, "rb").read()
    out = []
    pos = 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            break
        n, = struct.unpack_from("<Q", data, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                out.append(data[i + off:i + off + size])
        pos = i + 32
    return out


def main():
    pats = sys.argv[2:]
    for k, co in enumerate(code_objects(sys.argv[1])):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(co)
        notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name], capture_output=True,
                               text=True).stdout
        os.unlink(f.name)
        cur = {}
        for line in notes.splitlines():
            m = re.match(r"\s*-?\s*\.(\w+):\s*(.*)", line)
            if not m:
                continue
            key, val = m.group(1), m.group(2).strip()
            if key == "agpr_count":  # a kernel's block starts (keys in alphabetical order)
                cur = {"agpr": val}
            elif key in ("group_segment_fixed_size", "private_segment_fixed_size", "sgpr_count", "vgpr_count",
                         "vgpr_spill_count", "sgpr_spill_count"):
                cur[key] = val
            elif key == "name" and not val.endswith(".kd"):
                cur["name"] = val
            elif key == "wavefront_size" and "name" in cur:  # ... and ends
                val = cur["name"]
                if not pats or any(s in val for s in pats):
                    print(f"{val[:100]:100s} vgpr {cur.get('vgpr_count')} agpr {cur.get('agpr')} "
                          f"spill {cur.get('vgpr_spill_count')} scratch {cur.get('private_segment_fixed_size')} "
                          f"lds {cur.get('group_segment_fixed_size')}")
                cur = {}


if __name__ == "__main__":
    main()
