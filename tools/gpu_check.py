import sys, time, numpy as np
sys.path.insert(0, "mass-raytrace_amd"); sys.path.insert(0, ".")
import massrt, oracle
G = "tests/golden"
ctx = massrt.Context(0)
rng = np.random.default_rng(0)
for name in ["cornell", "sphere_grid", "cube_field"]:
    b = massrt.Builder(1).builtin(name, float(massrt.ASPECT_RATIO), G)
    ctx.upload(b)
    o = oracle.Scene(1).builtin(name, float(massrt.ASPECT_RATIO), G)
    # rays: camera-ish origins toward random targets
    n = 20000
    org = rng.uniform(-20, 20, (n, 3)).astype(np.float32); org[:,1] = np.abs(org[:,1]) + 1
    d = rng.normal(size=(n,3)).astype(np.float32)
    rays = np.concatenate([org, d], 1)
    gh = ctx.trace_rays(rays); oh = o.trace_rays(rays)
    print(name, "trace_rays equal:", np.array_equal(gh, oh), "hits", (gh[:,0]!=0).sum(), "mismatch rows", int((gh!=oh).any(1).sum()))
    W, H, spp = 64, 36, 4
    ctx.reset_counters(); o.reset_counters()
    t=time.time(); grgb, gb = ctx.render(W, H, 0, spp, seed=7, counters=True); gt=time.time()-t
    orgb, ob = o.render(W, H, 0, spp, seed=7, threads=8)
    rel = np.linalg.norm(grgb-orgb)/max(np.linalg.norm(orgb),1e-30)
    gc, oc = ctx.counters(), o.counters()
    print(" render bounces equal:", np.array_equal(gb, ob), "rgb rel L2", rel, "bitexact", np.array_equal(grgb, orgb), f"gpu {gt:.3f}s")
    print(" counters gpu", gc); print(" counters orc", {k:v for k,v in oc.items() if k!='alpha_taps'})
# throughput probe
b = massrt.Builder(1).builtin("sphere_grid", float(massrt.ASPECT_RATIO), G); ctx.upload(b)
for spp in [1, 8, 32]:
    ctx.render(1920, 1080, 0, 1, seed=1)
    t=time.time(); ctx.render(1920, 1080, 0, spp, seed=1); dt=time.time()-t
    print(f"sphere_grid 1080p spp={spp}: {dt:.3f}s  {1920*1080*spp/dt/1e6:.1f} Msamples/s")
