"""Static instruction counts of the JIT lane kernels in an ISA file written by
lane_isa.py: per kernel, VALU / SALU / memory instructions, lane read/write
(SGPR spill traffic), and the remarks' registers / scratch.
python scripts/isa_stats.py [/tmp/isa/lane_farmer]"""
import re
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa/lane_farmer"
s = open(base + ".s").read()
rem = open(base + ".remarks").read()
names = re.findall(r"^(phx_\w+):", s, re.M)
for name in names:
    m = re.search(r"^%s:.*?\n(.*?)^\.Lfunc_end" % name, s, re.S | re.M)
    lines = [l.strip() for l in m.group(1).split("\n")]
    ins = [l for l in lines if l and not l.startswith((".", ";")) and not l.endswith(":")]
    v = sum(1 for l in ins if l.startswith("v_"))
    sa = sum(1 for l in ins if l.startswith("s_"))
    mem = sum(1 for l in ins if l.startswith(("global_", "buffer_", "scratch_", "flat_")))
    rl = sum(1 for l in ins if "v_readlane" in l or "v_writelane" in l)
    f64 = sum(1 for l in ins if re.match(r"v_\w+_f64", l))
    print("%-20s ins %6d valu %6d (f64 %5d) salu %5d mem %4d lane-rw %4d" % (name, len(ins), v, f64, sa, mem, rl))
for blk in re.split(r"(?=remark: Function Name)", rem):
    m = re.search(r"Function Name: (\S+)", blk)
    if not m:
        continue
    vals = dict(re.findall(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", blk))
    print("%-20s %s" % (m.group(1), vals))
