"""Per-frame k_shade durations by level from a rocprofv3 SQLite kernel trace (tools/gpu_r5v49.sh, v50):
frames start at k_frame_start; frames 0-2 are unlit, 3-5 lit in tools/shade_lit_probe.py."""
import sqlite3,re,sys
db=sqlite3.connect(sys.argv[1])
rows=db.execute("select name, start, end from kernels order by start").fetchall()
def short(n):
    m=re.search(r'(k_[a-z_0-9]+(<[^>]*>)?)',n); return m.group(1) if m else n[:30]
frames=[];cur=None
for n,s,e in rows:
    k=short(n); d=(e-s)/1e3
    if k.startswith('k_frame_start'):
        cur=[];frames.append(cur)
    if cur is not None: cur.append((k,d))
for fi,f in enumerate(frames):
    sh=[round(d) for k,d in f if k.startswith('k_shade')]
    print("frame",fi,"total %.0f"%sum(d for k,d in f if not k.startswith(('k_lm','k_gr','k_sh_'))), "k_shade per level", sh)
