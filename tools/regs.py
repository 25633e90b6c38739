"""Per-kernel register / scratch / spill table from hipcc -Rpass-analysis=kernel-resource-usage
(compile-time check, no GPU).  python tools/regs.py [filter]  (builds conv.hip / kernels.hip device-only)"""
import os, re, subprocess, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(HERE, "inference-time-scaling-for-diffusion-models-beyond-scaling-denoising-steps_amd")
flt = sys.argv[1] if len(sys.argv) > 1 else ""
srcs = [a for a in sys.argv[2:]] or ["conv.hip"]
for s in srcs:
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(PKG, "csrc"),
           "-I", os.path.join(HERE, "include"), "-munsafe-fp-atomics", "--cuda-device-only", "-c",
           os.path.join(PKG, "csrc", s), "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"]
    if s == "conv.hip":
        cmd.append("-fno-slp-vectorize")
    r = subprocess.run(cmd, capture_output=True, text=True)
    cur = None
    rows = {}
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
        if m and cur:
            rows[cur][m.group(1).strip()] = int(m.group(2))
    for k, v in rows.items():
        if flt in k:
            print(f"{k[:70]:70s} vgpr {v.get('VGPRs',0):3d} agpr {v.get('AGPRs',0):3d} scratch {v.get('ScratchSize [bytes/lane]',0):4d} "
                  f"vspill {v.get('VGPRs Spill',0):3d} sspill {v.get('SGPRs Spill',0):3d} sgpr {v.get('SGPRs',0):3d} occ {v.get('Occupancy [waves/SIMD]',0)}")
