"""Pawn debugging (experiments only): GPU vs host core per scenario, single
launches and one batched launch, product library and libhtp_dbg.so (-DHTP_HA_DEBUG)."""
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from headland_trajectory_planning_amd import _native  # noqa: E402
import _ha_util as U  # noqa: E402
import _hostsim as H  # noqa: E402

probs = [U.scenario_pawn(s, n_obs=1 + s % 3) for s in range(16)]
host = H.as_dicts(H.hastar_host(probs))
for name in sys.argv[1:]:
    lib = _native.LIB_PATH if name == "base" else _native.LIB_PATH.replace("libhtp.so", f"libhtp_{name}.so")
    ctx = _native.Context(0, lib=_native.load(lib))
    for s, p in enumerate(probs):
        g = H.as_dicts(ctx.hastar(_native.HastarPacked([p])))[0]
        d = U.compare(host[s], g, exact=False)
        if d:
            print(f"{name} single seed {s}: {d[:4]}", flush=True)
    print(f"=== {name} batch", flush=True)
    g = H.as_dicts(ctx.hastar(_native.HastarPacked(probs)))
    for s in range(16):
        d = U.compare(host[s], g[s], exact=False)
        if d:
            print(f"{name} batch seed {s}: {d[:4]}", flush=True)
    print(f"=== {name} done", flush=True)
