"""Per-kernel register / scratch / LDS use of a built HIP object (gfx950).

    python tools/kres.py libpointmatcher_amd/build/pmx_grid.o [name-filter]

Unbundles the device code object with llvm-objdump --offloading into a temp
directory and reads the AMDGPU metadata notes (llvm-readelf --notes).
"""
import os, re, subprocess, sys, tempfile

B = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    obj = os.path.abspath(obj)
    with tempfile.TemporaryDirectory() as td:
        subprocess.run([f"{B}/llvm-objdump", "--offloading", obj], cwd=td, check=True,
                       stdout=subprocess.DEVNULL)
        # (objdump writes next to the input)
        dev = [f for f in os.listdir(os.path.dirname(obj)) if f.startswith(os.path.basename(obj) + ".0.hipv4")]
        out = []
        for f in dev:
            p = os.path.join(os.path.dirname(obj), f)
            txt = subprocess.run([f"{B}/llvm-readelf", "--notes", p], capture_output=True, text=True).stdout
            os.unlink(p)
            for h in os.listdir(os.path.dirname(obj)):
                if h.startswith(os.path.basename(obj) + ".0.host"):
                    os.unlink(os.path.join(os.path.dirname(obj), h))
            cur = {}
            for line in txt.splitlines():
                m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)$", line)
                if not m:
                    continue
                k, v = m.group(1), m.group(2).strip()
                if k in ("agpr_count", "group_segment_fixed_size", "private_segment_fixed_size", "sgpr_count",
                         "vgpr_count", "vgpr_spill_count", "sgpr_spill_count"):
                    cur[k] = int(v)
                elif k == "name":
                    cur["name"] = v
                elif k == "symbol" or k == "wavefront_size":
                    if "name" in cur and "vgpr_count" in cur:
                        pass
                if "name" in cur and "vgpr_count" in cur and "private_segment_fixed_size" in cur and \
                        "group_segment_fixed_size" in cur and "sgpr_count" in cur:
                    out.append(cur)
                    cur = {}
        return out


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    dem = lambda s: subprocess.run(["c++filt"], input=s, capture_output=True, text=True).stdout.strip()
    for k in kernels(sys.argv[1]):
        n = dem(k["name"])
        if flt in n:
            print(f"v{k['vgpr_count']:3d} a{k.get('agpr_count', 0):3d} s{k['sgpr_count']:3d} "
                  f"scr{k['private_segment_fixed_size']:5d} lds{k['group_segment_fixed_size']:6d}  {n[:150]}")
