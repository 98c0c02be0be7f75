#!/usr/bin/env python3
"""Build the generators of the BASELINE.json configs[4] mesh: a 60-3 km variable-resolution spherical
centroidal Voronoi tessellation with 835586 cells (the MPAS x20.835586 mesh's size and range), and
store them quantised to int32 per coordinate (mpas_dycore/data/x20.835586_generators.npz) so the GPU
box only triangulates (mesh.varres_from_generators).

Density (MPAS convention, cell spacing ~ rho^-1/4): rho = (1-g)/2 (tanh((beta-d)/alpha) + 1) + g,
g = 20^-4, beta = 9 deg, alpha = 3 deg, centred at (30N, 90W): integrating sqrt(rho) over the sphere
with 3 km hexagons in the refined disc gives 835714 cells, i.e. 3 km there and 60 km far away.

Construction (multilevel Lloyd): a 3266-generator SCVT of the same density (a Fibonacci lattice
remapped radially so that the point density is ~ sqrt(rho), relaxed by many Lloyd iterations), then
four refinements, each adding the midpoint of every Delaunay edge (N -> 4 N - 6: 3266 -> 13058 ->
52226 -> 208898 -> 835586) and relaxing again with density-weighted Lloyd iterations on the spherical
Delaunay triangulation, rebuilt every step.  Refinement keeps the coarse mesh's few pentagon /
heptagon defects, and each level only has to relax what the new points change.  Last, a few
rounds of opening the nearly co-circular generator quads Lloyd leaves at pentagon / heptagon pairs
(mesh._untangle_cocircular: a Voronoi edge shorter than 5 % of its cell distance) alternating with
Lloyd steps.  Result: 2.46-63.6 km, 597 pentagons, 585 heptagons, dvEdge / dcEdge >= 0.05.

    python tools/make_varres_mesh.py [--iters 300] [--out mpas-model_amd/mpas_dycore/data/...]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpas-model_amd"))

from mpas_dycore import mesh as M  # noqa: E402

NCELLS, CENTER, RADIUS_DEG, WIDTH_DEG, RATIO = 835586, (30.0, -90.0), 9.0, 3.0, 20.0


def radial_start(n):
    """Fibonacci points, each moved along its great circle from the centre so that the cumulative
    count inside distance d follows the integral of sqrt(rho) (point density ~ sqrt(rho))."""
    p = M._fibonacci_sphere(n)
    lat, lon = np.radians(CENTER[0]), np.radians(CENTER[1])
    zc = np.array([np.cos(lat) * np.cos(lon), np.cos(lat) * np.sin(lon), np.sin(lat)])
    rho = M.varres_density(CENTER, RADIUS_DEG, WIDTH_DEG, RATIO)
    d = np.linspace(0.0, np.pi, 400001)
    ray = np.cos(d)[:, None] * zc + np.sin(d)[:, None] * np.cross(zc, [0.0, 0.0, 1.0]) / np.linalg.norm(
        np.cross(zc, [0.0, 0.0, 1.0]))
    w = np.sqrt(rho(ray)) * np.sin(d)
    cdf = np.concatenate([[0.0], np.cumsum(0.5 * (w[1:] + w[:-1]) * np.diff(d))])
    cdf /= cdf[-1]
    d0 = np.arccos(np.clip(p @ zc, -1.0, 1.0))
    d1 = np.interp((1.0 - np.cos(d0)) / 2.0, cdf, d)
    t = p - (p @ zc)[:, None] * zc  # direction away from the centre
    t /= np.maximum(np.linalg.norm(t, axis=1), 1e-300)[:, None]
    return M._normalize(np.cos(d1)[:, None] * zc + np.sin(d1)[:, None] * t)


def quality(p):
    f = M._delaunay(p)
    vc = M._circumcenters(p, f)
    pairs = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
    face = np.concatenate([np.arange(len(f))] * 3)
    s = np.sort(pairs, axis=1)
    o = np.lexsort((s[:, 1], s[:, 0]))
    s, face = s[o], face[o]
    a, fa, fb = s[0::2], face[0::2], face[1::2]
    dv = np.linalg.norm(vc[fa] - vc[fb], axis=1)
    dc = np.linalg.norm(p[a[:, 0]] - p[a[:, 1]], axis=1)
    deg = np.bincount(f.ravel(), minlength=len(p))
    R = M.SPHERE_RADIUS / 1e3
    return dict(dc_min_km=float(dc.min() * R), dc_max_km=float(dc.max() * R), dv_over_dc_min=float((dv / dc).min()),
                n_small_dv=int((dv < 0.2 * dc).sum()), deg={int(k): int((deg == k).sum()) for k in np.unique(deg)})


def refine(p):
    """Add the normalised midpoint of every Delaunay edge: N -> 4 N - 6 generators."""
    f = M._delaunay(p)
    e = np.sort(np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]]), axis=1)
    e = np.unique(e, axis=0)
    return np.concatenate([p, M._normalize(p[e[:, 0]] + p[e[:, 1]])])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", default="600,200,80,40,30", help="Lloyd iterations per level, coarse to fine")
    ap.add_argument("--polish", type=int, default=3, help="rounds of untangling + 4 Lloyd steps at the end")
    ap.add_argument("--checkpoint", default="/tmp/varres_gen")
    ap.add_argument("--out", default=os.path.join(ROOT, "mpas-model_amd", "mpas_dycore", "data",
                                                  "x20.835586_generators.npz"))
    a = ap.parse_args()
    iters = [int(x) for x in a.iters.split(",")]
    rho = M.varres_density(CENTER, RADIUS_DEG, WIDTH_DEG, RATIO)
    n0 = (NCELLS + 510) // 256
    assert 256 * n0 - 510 == NCELLS
    p = radial_start(n0)
    t0 = time.time()
    for level, nit in enumerate(iters):
        if level:
            p = refine(p)
        for it in range(nit):
            p = M._lloyd_step(p, M._delaunay(p), rho)
            if len(p) > 200000 and (it + 1) % 10 == 0:
                print(f"level {level} ({len(p)}): iter {it + 1} {time.time() - t0:.0f} s", flush=True)
        np.save(f"{a.checkpoint}_{level}.npy", p)
        print(f"level {level}: {len(p)} generators, {nit} iterations, {time.time() - t0:.0f} s {quality(p)}",
              flush=True)
    assert len(p) == NCELLS
    for cyc in range(a.polish):
        p = M._untangle_cocircular(p, min_ratio=0.05, step=0.15, rounds=30)
        for _ in range(4):
            p = M._lloyd_step(p, M._delaunay(p), rho)
        print(f"polish {cyc + 1}: {quality(p)}", flush=True)
    p = M._untangle_cocircular(p, min_ratio=0.05, step=0.15, rounds=30)
    q = np.round(p * 2.0 ** 30).astype(np.int32)  # |x| <= 1: int32 with 2^-30 steps (~6 mm on Earth)
    np.savez_compressed(a.out, xyz_q30=q, center=np.array(CENTER), radius_deg=RADIUS_DEG, width_deg=WIDTH_DEG,
                        ratio=RATIO)
    print(f"wrote {a.out}: {quality(M._normalize(q / 2.0 ** 30))}", flush=True)


if __name__ == "__main__":
    main()
