"""Synthetic initial state and mesh-coefficient precompute for the dycore.

This is SURVEY.md §8(f) row 1 (the initial-state and mesh-coefficient pipeline),
restated in numpy so the GPU box (which never sees /root/reference) can build
the synthetic inputs of BASELINE.json's configs on its own:

* vertical grid and metrics       -- core_init_atmosphere/mpas_init_atm_cases.F:615-706
* Jablonowski-Williamson state    -- mpas_init_atm_cases.F:367-1160, with the
                                     reference's rebalance = .true. (the zonal wind
                                     geostrophically rebalanced on a 721-latitude
                                     grid, 720-838 and 1215-1312) or, with
                                     rebalance=False, the analytic JW wind (1005-1011)
* zb / zb3 terrain flux metrics   -- mpas_init_atm_cases.F:1045-1093
* deriv_two (quadratic LSQ fit)   -- core_init_atmosphere/mpas_atm_advection.F:21-394
* defc_a / defc_b                 -- core_init_atmosphere/mpas_atm_advection.F:744-946
* signs, zb_cell, kiteForCell     -- core_atmosphere/mpas_atm_core.F:987-1074
* adv_coefs compression           -- core_atmosphere/mpas_atm_core.F:1121-1266
* couple_coef_3rd_order           -- core_atmosphere/mpas_atm_core.F:1269-1288
* damping coefficients (dss)      -- core_atmosphere/mpas_atm_core.F:1077-1118
* mesh scaling                    -- core_atmosphere/mpas_atm_core.F:927-984
* inverses                        -- core_atmosphere/mpas_atm_core.F:339-353

These are *inputs* of the hot path; the oracle (the compiled reference Fortran)
and the HIP product both consume exactly the arrays produced here, so their
fidelity to the reference init affects realism, not parity.
"""
from __future__ import annotations

import os

import math

import numpy as np

from .reconstruct import init_reconstruct

from .mesh import _normalize, arc_length

# mpas_constants.F:25-36 (all promoted to double by -fdefault-real-8)
PII = 3.141592653589793
OMEGA = 7.29212e-5
GRAVITY = 9.80616
RGAS = 287.0
RV = 461.6
RVORD = RV / RGAS
CP = 7.0 * RGAS / 2.0
CV = CP - RGAS
P0 = 1.0e5

DEFAULT_CONFIG = dict(
    config_time_integration_order=2, config_dt=720.0, config_split_dynamics_transport=True,
    config_number_of_sub_steps=2, config_dynamics_split_steps=3,
    config_h_mom_eddy_visc2=0.0, config_h_mom_eddy_visc4=0.0, config_v_mom_eddy_visc2=0.0,
    config_h_theta_eddy_visc2=0.0, config_h_theta_eddy_visc4=0.0, config_v_theta_eddy_visc2=0.0,
    config_horiz_mixing="2d_smagorinsky", config_len_disp=120000.0, config_visc4_2dsmag=0.05,
    config_del4u_div_factor=10.0, config_scalar_advection=True, config_positive_definite=False,
    config_monotonic=True, config_coef_3rd_order=0.25, config_smagorinsky_coef=0.125,
    config_mix_full=True, config_epssm=0.1, config_smdiv=0.1, config_apvm_upwinding=0.5,
    config_h_ScaleWithMesh=True, config_zd=22000.0, config_xnutr=0.2, config_mpas_cam_coef=0.0,
    config_rayleigh_damp_u=False, config_rayleigh_damp_u_timescale_days=5.0,
    config_number_rayleigh_damp_u_levels=6,
)  # Registry.xml:56-290 defaults


def vertical_grid(K: int, zt: float = 45000.0):
    """mpas_init_atm_cases.F:615-678 (uniform dzeta, str=1.5 stretching)."""
    nz1, nz = K, K + 1
    dz = zt / float(nz1)
    k = np.arange(nz)
    sh = _pow(k * dz / zt, 1.5)
    zw = k * dz
    ah = 1.0 - _ipow(np.cos(0.5 * PII * k * dz / zt), 6)
    dzw = zw[1:] - zw[:-1]
    rdzw = 1.0 / dzw
    dzu = np.zeros(nz1)
    rdzu = np.zeros(nz1)
    fzp = np.zeros(nz1)
    fzm = np.zeros(nz1)
    dzu[1:] = 0.5 * (dzw[1:] + dzw[:-1])
    rdzu[1:] = 1.0 / dzu[1:]
    fzp[1:] = 0.5 * dzw[1:] / dzu[1:]
    fzm[1:] = 0.5 * dzw[:-1] / dzu[1:]
    cof1 = (2.0 * dzu[1] + dzu[2]) / (dzu[1] + dzu[2]) * dzw[0] / dzu[1]
    cof2 = dzu[1] / (dzu[1] + dzu[2]) * dzw[0] / dzu[2]
    cf1 = fzp[1] + cof1
    cf2 = fzm[1] - cof1 - cof2
    cf3 = cof2
    return dict(zt=zt, sh=sh, zw=zw, ah=ah, dzw=dzw, rdzw=rdzw, dzu=dzu, rdzu=rdzu,
                fzp=fzp, fzm=fzm, cf1=cf1, cf2=cf2, cf3=cf3)


def _jw_hx(phi, r_earth):
    u0 = 35.0
    etavs = (1.0 - 0.252) * PII / 2.0
    ce15 = _pow(np.cos(etavs), 1.5)
    sp, cp = _sincos(phi)  # one sincos(phi) for the statement (606-611)
    return (u0 / GRAVITY * ce15
            * ((-2.0 * _ipow(sp, 6) * (cp ** 2 + 1.0 / 3.0) + 10.0 / 63.0)
               * u0 * ce15
               + (1.6 * _ipow(cp, 3) * (sp ** 2 + 2.0 / 3.0) - PII / 4.0) * r_earth * OMEGA))


# ---- the reference's spherical geometry (core_init_atmosphere/mpas_atm_advection.F:397-537),
# elementwise over arrays of points (..., 3); same expressions, same evaluation order.
# asin / acos go through the C library (math.asin / math.acos), as the compiled Fortran does:
# numpy's own arcsin / arccos differ from it in the last bit for ~8 % of arguments, which the
# ill-conditioned least-squares fits of deriv_two amplify to ~1e-8.
_LIBM_ASIN = np.frompyfunc(math.asin, 1, 1)
_LIBM_ACOS = np.frompyfunc(math.acos, 1, 1)


_LIBM_POW = np.frompyfunc(math.pow, 2, 1)
_LIBM_EXP = np.frompyfunc(math.exp, 1, 1)
_LIBM_TAN = np.frompyfunc(math.tan, 1, 1)

# The same C library functions looped in C (csrc/host_libm.c -> csrc/libmpas_host.so, built with
# the dycore): the math.* calls above one element per Python call take minutes at 835586 cells.
# Same library, same results; without the built helper the math.* loops run.
_HOST = None
try:
    import ctypes as _C
    _HOST = _C.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc",
                                 "libmpas_host.so"))
    for _f in ("hl_exp", "hl_asin", "hl_acos", "hl_tan"):
        getattr(_HOST, _f).argtypes = [_C.c_void_p, _C.c_void_p, _C.c_int64]
    _HOST.hl_pow_s.argtypes = [_C.c_void_p, _C.c_double, _C.c_void_p, _C.c_int64]
    _HOST.hl_sincos.argtypes = [_C.c_void_p, _C.c_void_p, _C.c_void_p, _C.c_int64]
except (OSError, AttributeError) as _e:  # not built, or a stale build without one of the helpers
    import warnings as _w
    _w.warn(f"mpas_dycore.init_atm: csrc/libmpas_host.so unusable ({_e}); the case builder falls back to "
            "numpy / math, whose sin, cos, exp, tan and pow differ from the compiled reference's C library in "
            "the last bit for some arguments (the JW state, deriv_two and defc are then not the reference's "
            "bits; rebuild with __graft_entry__.build())", RuntimeWarning, stacklevel=2)
    _HOST = None


def host_libm_loaded() -> bool:
    """True when the case builder uses the C library's functions (csrc/libmpas_host.so), i.e. its
    initial states are the compiled reference's bits (cases record it as case["host_libm"])."""
    return _HOST is not None


def _sincos(x):
    """(sin x, cos x) as the compiled reference gets them where it evaluates both of one argument in
    one place: amdflang -O2 merges the pair into one call of the C library's sincos(), which differs
    from separate sin / cos in the last bit for ~0.06 % of arguments (measured with the same
    compiler here).  Without the built helper, numpy's sin / cos (the separate functions' values)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    if _HOST is None:
        return np.sin(x), np.cos(x)
    sn, cs = np.empty_like(x), np.empty_like(x)
    _HOST.hl_sincos(x.ctypes.data, sn.ctypes.data, cs.ctypes.data, x.size)
    return sn, cs


def _host1(fn, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    fn(x.ctypes.data, out.ctypes.data, x.size)
    return out


# The JW initial state follows the compiled reference's arithmetic (checked against amdflang's
# lowering): x**n with an integer n is the product x*x*...*x from the left, x**r with a real r and
# exp / tan / asin are the C library's; numpy's own exp, tan and pow differ from it in the last
# bit for about 5 % of arguments (sin, cos, sqrt agree).
def _ipow(x, n):
    r = x
    for _ in range(n - 1):
        r = r * x
    return r


def _exp(x):
    if _HOST is not None:
        return _host1(_HOST.hl_exp, x)
    return np.asarray(_LIBM_EXP(np.asarray(x, dtype=np.float64)), dtype=np.float64)


def _tan(x):
    if _HOST is not None:
        return _host1(_HOST.hl_tan, x)
    return np.asarray(_LIBM_TAN(np.asarray(x, dtype=np.float64)), dtype=np.float64)


def _pow(x, y):
    """Fortran x**y with a real constant exponent, as the compiled reference evaluates it: the
    compiler turns **0.75 into sqrt(x) * sqrt(sqrt(x)); **0.25 and the other exponents call the C
    library's pow (each checked bit for bit against the reference build: meshScalingDel4 / Del2,
    dss on the variable-resolution mesh)."""
    x = np.asarray(x, dtype=np.float64)
    if y == 0.75:
        return np.sqrt(x) * np.sqrt(np.sqrt(x))
    if _HOST is not None:
        x = np.ascontiguousarray(x)
        out = np.empty_like(x)
        _HOST.hl_pow_s(x.ctypes.data, float(y), out.ctypes.data, x.size)
        return out
    return np.asarray(_LIBM_POW(x, float(y)), dtype=np.float64)


def _asin(x):
    if _HOST is not None:
        return _host1(_HOST.hl_asin, x)
    return np.asarray(_LIBM_ASIN(np.asarray(x, dtype=np.float64)), dtype=np.float64)


def _acos(x):
    if _HOST is not None:
        return _host1(_HOST.hl_acos, x)
    return np.asarray(_LIBM_ACOS(np.asarray(x, dtype=np.float64)), dtype=np.float64)

def _ref_arc_length(a, b):
    """arc_length (490-510)."""
    cx, cy, cz = b[..., 0] - a[..., 0], b[..., 1] - a[..., 1], b[..., 2] - a[..., 2]
    r = np.sqrt(a[..., 0] * a[..., 0] + a[..., 1] * a[..., 1] + a[..., 2] * a[..., 2])
    c = np.sqrt(cx * cx + cy * cy + cz * cz)
    return r * 2.0 * _asin(c / (2.0 * r))


def _ref_sphere_angle(a, b, c):
    """sphere_angle (403-447): the angle between arcs AB and AC."""
    la = _ref_arc_length(b, c)
    lb = _ref_arc_length(a, c)
    lc = _ref_arc_length(a, b)
    abx, aby, abz = b[..., 0] - a[..., 0], b[..., 1] - a[..., 1], b[..., 2] - a[..., 2]
    acx, acy, acz = c[..., 0] - a[..., 0], c[..., 1] - a[..., 1], c[..., 2] - a[..., 2]
    dx = (aby * acz) - (abz * acy)
    dy = -((abx * acz) - (abz * acx))
    dz = (abx * acy) - (aby * acx)
    sp = 0.5 * (la + lb + lc)
    with np.errstate(invalid="ignore", divide="ignore"):
        q = (np.sin(sp - lb) * np.sin(sp - lc)) / (np.sin(lb) * np.sin(lc))
    sin_angle = np.sqrt(np.minimum(1.0, np.maximum(0.0, np.nan_to_num(q, nan=0.0))))
    ang = 2.0 * _asin(np.maximum(np.minimum(sin_angle, 1.0), -1.0))
    return np.where((dx * a[..., 0] + dy * a[..., 1] + dz * a[..., 2]) >= 0.0, ang, -ang)


def _ref_plane_angle_z(bx, by, cx, cy):
    """plane_angle (457-485) with A = 0, B = (bx, by, 0), C = (cx, cy, 0), normal (0, 0, 1)."""
    mab = np.sqrt(bx * bx + by * by + 0.0 * 0.0)
    mac = np.sqrt(cx * cx + cy * cy + 0.0 * 0.0)
    dz = (bx * cy) - (by * cx)
    cos_angle = (bx * cx + by * cy + 0.0 * 0.0) / (mab * mac)
    ang = _acos(np.maximum(np.minimum(cos_angle, 1.0), -1.0))
    return np.where(dz >= 0.0, ang, -ang)


def _ref_arc_bisect(a, b):
    """arc_bisect (520-537)."""
    r = np.sqrt(a[..., 0] * a[..., 0] + a[..., 1] * a[..., 1] + a[..., 2] * a[..., 2])
    c = 0.5 * (a + b)
    d = np.sqrt(c[..., 0] * c[..., 0] + c[..., 1] * c[..., 1] + c[..., 2] * c[..., 2])
    return r[..., None] * c / d[..., None]


def _ref_migs(a):
    """MIGS / ELGS (642-740): inverse by partial-pivoting Gaussian elimination, batched over the
    leading axis; same pivot choice (first largest scaled element) and update order."""
    if a.shape[0] > 8192:  # independent systems: batches that stay in cache
        return np.concatenate([_ref_migs(a[i:i + 8192]) for i in range(0, a.shape[0], 8192)])
    a = a.copy()
    nb, n, _ = a.shape
    rows = np.arange(nb)
    indx = np.tile(np.arange(n), (nb, 1))
    cs = np.max(np.abs(a), axis=2)                     # rescaling factor of every row
    for j in range(n - 1):
        pi1 = np.zeros(nb)
        k = np.full(nb, j)
        for i in range(j, n):
            pv = np.abs(a[rows, indx[:, i], j]) / cs[rows, indx[:, i]]
            take = pv > pi1
            pi1 = np.where(take, pv, pi1)
            k = np.where(take, i, k)
        tj = indx[:, j].copy()
        indx[:, j] = indx[rows, k]
        indx[rows, k] = tj
        for i in range(j + 1, n):
            ri, rj = indx[:, i], indx[:, j]
            pj = a[rows, ri, j] / a[rows, rj, j]
            a[rows, ri, j] = pj
            for kk in range(j + 1, n):
                a[rows, ri, kk] = a[rows, ri, kk] - pj * a[rows, rj, kk]
    b = np.zeros((nb, n, n))
    b[:, np.arange(n), np.arange(n)] = 1.0
    for i in range(n - 1):
        for j in range(i + 1, n):
            rj, ri = indx[:, j], indx[:, i]
            for kk in range(n):
                b[rows, rj, kk] = b[rows, rj, kk] - a[rows, rj, i] * b[rows, ri, kk]
    x = np.zeros((nb, n, n))
    for i in range(n):
        rn = indx[:, n - 1]
        x[:, n - 1, i] = b[rows, rn, i] / a[rows, rn, n - 1]
        for j in range(n - 2, -1, -1):
            rj = indx[:, j]
            v = b[rows, rj, i]
            for kk in range(j + 1, n):
                v = v - a[rows, rj, kk] * x[:, kk, i]
            x[:, j, i] = v / a[rows, rj, j]
    return x


def _matmul_seq(x, y):
    """Fortran matmul with the sum over the inner index taken in order from zero (batched)."""
    out = np.zeros((x.shape[0], x.shape[1], y.shape[2]))
    for k in range(x.shape[2]):
        out = out + x[:, :, k:k + 1] * y[:, k:k + 1, :]
    return out


def _ref_local_polygon(c, pts, R):
    """The tangent-plane coordinates both initialisations build (mpas_atm_advection.F:132-179,
    823-874): theta_abs, the angles between consecutive points seen from the centre (thetav),
    and the points' great-circle distances; pts (nc, n-1, 3) around centres c (nc, 3), unit sphere."""
    nc, m = pts.shape[0], pts.shape[1]
    pole = np.broadcast_to(np.array([0.0, 0.0, 1.0]), c.shape)
    theta_abs = np.where(c[:, 2] == 1.0, PII / 2.0, PII / 2.0 - _ref_sphere_angle(c, pts[:, 0], pole))
    nxt = pts[:, (np.arange(m) + 1) % m]               # ip2 wraps to the first point
    cb = np.broadcast_to(c[:, None, :], pts.shape)
    thetav = _ref_sphere_angle(cb, pts, nxt)
    dl = R * _ref_arc_length(cb, pts)
    return theta_abs, thetav, dl


def deriv_two_inputs(m):
    """The transcendental half of atm_initialize_advection_rk (mpas_atm_advection.F:21-394,
    polynomial_order = 2, on a sphere), per cell and edgesOnCell slot: the tangent-plane coordinates
    xp / yp of the neighbour cellsOnCell(i) (132-181) and sin / cos of the angle thetae of the edge's
    normal direction (303-315, 334-335 / 347-348), from the C library's asin / sin / cos / sincos as the
    compiled reference takes them.  Returns (xp, yp, sin_the, cos_the), each (nCells, maxEdges), zero
    beyond nEdgesOnCell: what deriv_two_fit (host) or mpas_dyc_init_deriv_two (device) turn into
    deriv_two."""
    nC, R = m["nCells"], m["sphere_radius"]
    xc = np.stack([m["xCell"], m["yCell"], m["zCell"]], 1) / R
    xv = np.stack([m["xVertex"], m["yVertex"], m["zVertex"]], 1) / R
    nEoC, coc, eoc, voe = m["nEdgesOnCell"], m["cellsOnCell"], m["edgesOnCell"], m["verticesOnEdge"]
    out = [np.zeros((nC, m["maxEdges"])) for _ in range(4)]
    for ne in np.unique(nEoC):
        cells = np.nonzero(nEoC == ne)[0]
        c = xc[cells]
        nb = xc[coc[cells, :ne]]
        theta_abs, thetav, dl = _ref_local_polygon(c, nb, R)
        thetat = np.empty((len(cells), ne))
        thetat[:, 0] = theta_abs                      # x direction along the longitude line (176)
        for i in range(1, ne):
            thetat[:, i] = thetat[:, i - 1] + thetav[:, i - 1]
        st_, ct_ = _sincos(thetat)  # 180-181: cos and sin of thetat(i) in one loop body
        out[0][cells, :ne] = ct_ * dl
        out[1][cells, :ne] = st_ * dl
        for i in range(ne):
            e = eoc[cells, i]
            mid = _ref_arc_bisect(xv[voe[e, 0]], xv[voe[e, 1]])
            the = _ref_sphere_angle(c, nb[:, i], mid) + thetat[:, i]
            out[2][cells, i], out[3][cells, i] = _sincos(the)  # 334-335 / 347-348
    return tuple(out)


def deriv_two_fit(m, xp_all, yp_all, sin_all, cos_all):
    """The arithmetic half (the host path; csrc/model_init.hip k_mi_deriv_two is the device one): per
    cell the weighted least-squares quadratic through the cell and its neighbours (amatrix 215-226,
    poly_fit_2 with MIGS, 567-741), and its second derivative along each edge's normal direction
    (327-358)."""
    nE = m["nEdges"]
    nEoC, eoc, coe = m["nEdgesOnCell"], m["edgesOnCell"], m["cellsOnEdge"]
    d2 = np.zeros((nE, 2, 15))
    for ne in np.unique(nEoC):
        cells = np.nonzero(nEoC == ne)[0]
        n = ne + 1
        xp, yp = xp_all[cells, :ne], yp_all[cells, :ne]
        a = np.zeros((len(cells), n, 6))
        a[:, 0, 0] = 1.0
        a[:, 1:, 0] = 1.0
        a[:, 1:, 1] = xp
        a[:, 1:, 2] = yp
        a[:, 1:, 3] = xp * xp
        a[:, 1:, 4] = xp * yp
        a[:, 1:, 5] = yp * yp
        at = np.transpose(a, (0, 2, 1))               # poly_fit_2 (567-614) with unit weights
        ath = _matmul_seq(at, np.broadcast_to(np.eye(n), (len(cells), n, n)))
        b = _matmul_seq(_ref_migs(_matmul_seq(ath, a)), ath)   # (nc, 6, n)
        for i in range(ne):
            e = eoc[cells, i]
            sin2t, cos2t = sin_all[cells, i], cos_all[cells, i]
            costsint = cos2t * sin2t
            cos2t, sin2t = cos2t * cos2t, sin2t * sin2t
            val = 2. * cos2t[:, None] * b[:, 3, :] + 2. * costsint[:, None] * b[:, 4, :] \
                + 2. * sin2t[:, None] * b[:, 5, :]
            side = np.where(coe[e, 0] == cells, 0, 1)
            d2[e, side, :n] = val
    return d2


def compute_deriv_two(m):
    """deriv_two, as atm_initialize_advection_rk computes it (mpas_atm_advection.F:21-394,
    polynomial_order = 2, on a sphere): per cell a weighted least-squares quadratic through the
    cell and its neighbours (poly_fit_2 with MIGS), the fit's second derivative along each edge's
    normal direction.  deriv_two[e, side, j]: side 0 when the cell is cellsOnEdge(1, e); j = 0 the
    cell itself, j = i + 1 its neighbour cellsOnCell(i)."""
    return deriv_two_fit(m, *deriv_two_inputs(m))


def compute_defc(m):
    """Deformation weights defc_a / defc_b as atm_initialize_deformation_weights computes them
    (mpas_atm_advection.F:744-937, on a sphere): the cell polygon in the tangent plane, each side's
    direction from theta_abs plus the turning angles (plane_angle), side length over cell area."""
    nC, R = m["nCells"], m["sphere_radius"]
    xc = np.stack([m["xCell"], m["yCell"], m["zCell"]], 1) / R
    xv = np.stack([m["xVertex"], m["yVertex"], m["zVertex"]], 1) / R
    nEoC, voc, eoc, coe = m["nEdgesOnCell"], m["verticesOnCell"], m["edgesOnCell"], m["cellsOnEdge"]
    defc_a = np.zeros((nC, m["maxEdges"]))
    defc_b = np.zeros((nC, m["maxEdges"]))
    for ne in np.unique(nEoC):
        cells = np.nonzero(nEoC == ne)[0]
        c = xc[cells]
        vv = xv[voc[cells, :ne]]
        theta_abs, thetav, dl = _ref_local_polygon(c, vv, R)
        th = np.empty((len(cells), ne))
        th[:, 0] = 0.0                                # 872: x direction towards the first vertex
        for i in range(1, ne):
            th[:, i] = th[:, i - 1] + thetav[:, i - 1]
        sth, cth = _sincos(th)  # 877-880: one sincos per thetat(i)
        xp, yp = cth * dl, sth * dl
        ip1 = (np.arange(ne) + 1) % ne
        thetat = np.empty((len(cells), ne))
        thetat[:, 0] = theta_abs                      # 894
        for i in range(1, ne):
            j = ip1[i]
            thetat[:, i] = _ref_plane_angle_z(xp[:, i] - xp[:, i - 1], yp[:, i] - yp[:, i - 1],
                                              xp[:, j] - xp[:, i], yp[:, j] - yp[:, i]) + thetat[:, i - 1]
        area = np.zeros(len(cells))
        for i in range(ne):                           # 907-914, summed in order
            j = ip1[i]
            area = area + 0.25 * (xp[:, i] + xp[:, j]) * (yp[:, j] - yp[:, i]) \
                - 0.25 * (yp[:, i] + yp[:, j]) * (xp[:, j] - xp[:, i])
        for i in range(ne):
            j = ip1[i]
            dls = np.sqrt((xp[:, j] - xp[:, i]) ** 2 + (yp[:, j] - yp[:, i]) ** 2)
            st, ct = _sincos(thetat[:, i])  # 923-925
            sint2, cost2, sint_cost = st * st, ct * ct, st * ct
            a = dls * (cost2 - sint2) / area
            b = dls * 2. * sint_cost / area
            flip = coe[eoc[cells, i], 0] != cells
            defc_a[cells, i] = np.where(flip, -a, a)
            defc_b[cells, i] = np.where(flip, -b, b)
    return defc_a, defc_b


def adv_coef_compression(m, d2):
    """mpas_atm_core.F:1154-1264, vectorised over edges."""
    nE, maxE = m["nEdges"], m["maxEdges"]
    coe, coc, nEoC, dc, dv = m["cellsOnEdge"], m["cellsOnCell"], m["nEdgesOnCell"], m["dcEdge"], m["dvEdge"]
    c1, c2 = coe[:, 0], coe[:, 1]
    lst = -np.ones((nE, 15), dtype=np.int64)
    lst[:, 0], lst[:, 1] = c1, c2
    n = np.full(nE, 2)
    ar = np.arange(nE)
    for i in range(maxE):
        cc = coc[c1, i]
        add = (i < nEoC[c1]) & (cc != c2)
        lst[ar[add], n[add]] = cc[add]
        n = n + add
    for i in range(maxE):
        cc = coc[c2, i]
        valid = i < nEoC[c2]
        present = np.any(lst == cc[:, None], axis=1)
        add = valid & ~present
        lst[ar[add], n[add]] = cc[add]
        n = n + add
    coef = np.zeros((nE, 15))
    coef3 = np.zeros((nE, 15))

    def jpos(cell):
        return np.argmax(lst == cell[:, None], axis=1)

    j = jpos(c1)
    coef[ar, j] += d2[:, 0, 0]
    coef3[ar, j] += d2[:, 0, 0]
    for i in range(maxE):
        v = i < nEoC[c1]
        j = jpos(coc[c1, i])
        coef[ar[v], j[v]] += d2[v, 0, i + 1]
        coef3[ar[v], j[v]] += d2[v, 0, i + 1]
    j = jpos(c2)
    coef[ar, j] += d2[:, 1, 0]
    coef3[ar, j] -= d2[:, 1, 0]
    for i in range(maxE):
        v = i < nEoC[c2]
        j = jpos(coc[c2, i])
        coef[ar[v], j[v]] += d2[v, 1, i + 1]
        coef3[ar[v], j[v]] -= d2[v, 1, i + 1]
    coef = -(dc[:, None] ** 2) * coef / 12.0
    coef3 = -(dc[:, None] ** 2) * coef3 / 12.0
    coef[ar, jpos(c1)] += 0.5
    coef[ar, jpos(c2)] += 0.5
    coef *= dv[:, None]
    coef3 *= dv[:, None]
    mask = np.arange(15)[None, :] < n[:, None]
    return n, np.where(mask, lst, -1), np.where(mask, coef, 0.0), np.where(mask, coef3, 0.0)


def build_case(m: dict, K: int = 26, ns: int = 1, moist: bool = False, config: dict | None = None,
               init_case: int = 2, rebalance: bool = True) -> dict:
    """Build every mesh/state/diag input array of the dycore for the JW case.

    ``rebalance`` (default): the zonal wind as the reference computes it (its parameter rebalance =
    .true., mpas_init_atm_cases.F:440): the JW wind on a 721-point latitude grid, rebalanced
    geostrophically (init_atm_recompute_geostrophic_wind) and integrated over each edge's
    latitude span (init_atm_calc_flux_zonal).  False: the analytic JW wind (1005-1011).
    Returns a flat dict keyed by MPAS field name (0-based index arrays, element-major
    (n, K) float arrays, i.e. the transpose of the Fortran (K, n) layout)."""
    cfg = dict(DEFAULT_CONFIG)
    if config:
        cfg.update(config)
    nC, nE, nV, R = m["nCells"], m["nEdges"], m["nVertices"], m["sphere_radius"]
    vg = vertical_grid(K)
    nz1, nz = K, K + 1
    lat = m["latCell"]
    coe, voe = m["cellsOnEdge"], m["verticesOnEdge"]
    c1, c2 = coe[:, 0], coe[:, 1]

    # ---- metrics (mpas_init_atm_cases.F:603-696)
    hx = _jw_hx(lat, R)
    zgrid = (1.0 - vg["ah"])[None, :] * (vg["sh"][None, :] * (vg["zt"] - hx[:, None]) + hx[:, None]) \
        + vg["ah"][None, :] * vg["sh"][None, :] * vg["zt"]                          # (nC, K+1)
    zz = (vg["zw"][1:] - vg["zw"][:-1])[None, :] / (zgrid[:, 1:] - zgrid[:, :-1])   # (nC, K)
    zxu = 0.5 * (zgrid[c2, :-1] - zgrid[c1, :-1] + zgrid[c2, 1:] - zgrid[c1, 1:]) / m["dcEdge"][:, None]

    # ---- JW thermodynamic state (mpas_init_atm_cases.F:839-958), column-independent:
    # computed over cache-sized chunks of cells with level-major work arrays.
    u0 = 35.0
    ppb = np.empty((nC, nz1))
    pp = np.empty((nC, nz1))
    rb = np.empty((nC, nz1))
    rr = np.empty((nC, nz1))
    tb = np.empty((nC, nz1))
    t = np.empty((nC, nz1))
    qv = np.empty((nC, nz1))
    CH = 2048
    chunks = [slice(c0, min(nC, c0 + CH)) for c0 in range(0, nC, CH)]
    nproc = min(16, os.cpu_count() or 1, len(chunks))
    if nproc > 1 and nC >= 20000:
        import concurrent.futures as cf
        import multiprocessing as mp
        with cf.ProcessPoolExecutor(nproc, mp_context=mp.get_context("fork")) as ex:
            results = list(ex.map(_jw_columns, [lat[sl] for sl in chunks], [zgrid[sl] for sl in chunks],
                                  [zz[sl] for sl in chunks], [vg] * len(chunks), [R] * len(chunks),
                                  [moist] * len(chunks)))
    else:
        results = [_jw_columns(lat[sl], zgrid[sl], zz[sl], vg, R, moist) for sl in chunks]
    for sl, r in zip(chunks, results):
        for a, b in zip((ppb, pp, rb, rr, tb, t, qv), r):
            a[sl] = b.T
    rho_zz = rb + rr
    fzp, fzm = vg["fzp"], vg["fzm"]

    # ---- wind (analytic JW flux, mpas_init_atm_cases.F:974-1019)
    latV = m["latVertex"]
    lat1, lat2 = latV[voe[:, 0]], latV[voe[:, 1]]
    flux = (0.5 * (lat2 - lat1) - 0.125 * (np.sin(4.0 * lat2) - np.sin(4.0 * lat1))) * R / m["dvEdge"]
    if init_case == 2:
        lat_pert, lon_pert = 40.0 * PII / 180.0, 20.0 * PII / 180.0
        le, lo = m["latEdge"], m["lonEdge"]
        # sphere_distance(latEdge, lonEdge, lat_pert, lon_pert, 1) (mpas_init_atm_static.F:1314-1328)
        arg1 = np.sqrt(np.sin(0.5 * (lat_pert - le)) ** 2 + np.cos(le) * np.cos(lat_pert) * np.sin(0.5 * (lon_pert - lo)) ** 2)
        r_pert = 2.0 * 1.0 * _asin(arg1) / 0.1
        u_pert = 1.0 * _exp(-r_pert ** 2) * (lat2 - lat1) * R / m["dvEdge"]
    else:
        u_pert = np.zeros(nE)
    if rebalance:
        u = u0 * _jw_flux_zonal(lat1, lat2, m["dvEdge"], R, vg, moist) / (0.5 * (rb[c1] + rb[c2] + rr[c1] + rr[c2])) \
            + u_pert[:, None]
    else:
        etavs = (0.5 * (ppb[c1] + ppb[c2] + pp[c1] + pp[c2]) / P0 - 0.252) * PII / 2.0
        u = u0 * flux[:, None] * _pow(np.cos(etavs), 1.5) + u_pert[:, None]
    ru = 0.5 * (rho_zz[c1] + rho_zz[c2]) * u

    # 1024-1036: 2 omega (-cos(lon) cos(lat) sin(alpha) + sin(lat) cos(alpha)) with alpha_grid = 0 is
    # 2 omega sin(lat), the sine from the statement's one sincos(lat)
    fEdge = 2.0 * OMEGA * _sincos(m["latEdge"])[0]
    fVertex = 2.0 * OMEGA * _sincos(m["latVertex"])[0]

    # ---- deriv_two, zb/zb3 (mpas_init_atm_cases.F:1045-1093, theta_adv_order = 3)
    d2 = m["deriv_two"] if "deriv_two" in m else compute_deriv_two(m)  # an init file may carry it
    nEoC, coc, eoc = m["nEdgesOnCell"], m["cellsOnCell"], m["edgesOnCell"]
    d2c1 = np.empty((nE, nz))
    d2c2 = np.empty((nE, nz))
    for e0 in range(0, nE, 32768):  # edge batches that stay in cache; per element the same sums
        s_ = slice(e0, min(nE, e0 + 32768))
        a1_, a2_ = c1[s_], c2[s_]
        x1 = d2[s_, 0, 0][:, None] * zgrid[a1_]
        x2 = d2[s_, 1, 0][:, None] * zgrid[a2_]
        for i in range(m["maxEdges"]):
            v1 = (i < nEoC[a1_])[:, None]
            v2 = (i < nEoC[a2_])[:, None]
            x1 = x1 + np.where(v1, d2[s_, 0, i + 1][:, None] * zgrid[coc[a1_, i]], 0.0)
            x2 = x2 + np.where(v2, d2[s_, 1, i + 1][:, None] * zgrid[coc[a2_, i]], 0.0)
        d2c1[s_] = x1
        d2c2[s_] = x2
    dcE = m["dcEdge"][:, None]
    z_edge = 0.5 * (zgrid[c1] + zgrid[c2]) - dcE ** 2 * (d2c1 + d2c2) / 12.0
    z_edge3 = -dcE ** 2 * (d2c1 - d2c2) / 12.0
    dv = m["dvEdge"][:, None]
    a1, a2 = m["areaCell"][c1][:, None], m["areaCell"][c2][:, None]
    zb = np.zeros((nE, 2, nz))
    zb3 = np.zeros((nE, 2, nz))
    zb[:, 0, :nz1] = ((z_edge - zgrid[c1]) * dv / a1)[:, :nz1]
    zb[:, 1, :nz1] = ((z_edge - zgrid[c2]) * dv / a2)[:, :nz1]
    zb3[:, 0, :nz1] = (z_edge3 * dv / a1)[:, :nz1]
    zb3[:, 1, :nz1] = (z_edge3 * dv / a2)[:, :nz1]

    # ---- rw / w from terrain (mpas_init_atm_cases.F:1096-1126)
    coef3 = cfg["config_coef_3rd_order"]
    rw = np.zeros((nC, nz))
    # the reference adds the edges' contributions in edge order (1103-1118): per cell, its edges in
    # ascending order, as cellsOnEdge(2) +A -B or as cellsOnEdge(1) -C +D
    eoc_sorted = np.sort(np.where(np.arange(m["maxEdges"])[None, :] < nEoC[:, None], eoc, nE), axis=1)
    for k0 in range(1, nz1, 8):  # 8 levels at a time, each level's expressions as written per k
        ks = np.arange(k0, min(nz1, k0 + 8))
        fl = fzm[ks] * ru[:, ks] + fzp[ks] * ru[:, ks - 1]
        z2 = fzm[ks] * zz[c2[:, None], ks] + fzp[ks] * zz[c2[:, None], ks - 1]
        z1 = fzm[ks] * zz[c1[:, None], ks] + fzp[ks] * zz[c1[:, None], ks - 1]
        sg = np.copysign(1.0, ru[:, ks])
        a2, b2 = z2 * zb[:, 1, ks] * fl, sg * coef3 * z2 * zb3[:, 1, ks] * fl
        a1, b1 = z1 * zb[:, 0, ks] * fl, sg * coef3 * z1 * zb3[:, 0, ks] * fl
        x = np.zeros((nC, len(ks)))
        for j in range(m["maxEdges"]):
            e = eoc_sorted[:, j]
            ok = e < nE
            ee = np.where(ok, e, 0)
            second = (c2[ee] == np.arange(nC))[:, None]
            okc = ok[:, None]
            x = np.where(okc & second, (x + a2[ee]) - b2[ee], np.where(okc, (x - a1[ee]) + b1[ee], x))
        rw[:, ks] = x
    w = np.zeros((nC, nz))
    w[:, 1:nz1] = rw[:, 1:nz1] / (fzp[1:] * rho_zz[:, :-1] + fzm[1:] * rho_zz[:, 1:])

    rho = rho_zz * zz
    theta = t / (1.0 + 1.61 * qv)

    scalars = np.zeros((nC, nz1, ns))
    if ns >= 1:
        scalars[:, :, 0] = qv
    if ns > 1:
        # smooth positive blobs so the monotonic limiter is exercised
        xc = np.stack([m["xCell"], m["yCell"], m["zCell"]], 1) / R
        rng = np.random.default_rng(20250202)
        for s in range(1, ns):
            ctr = _normalize(rng.normal(size=3))
            d = arc_length(xc, np.broadcast_to(ctr, xc.shape))
            prof = np.exp(-((np.arange(nz1) - nz1 * 0.3) / (0.15 * nz1)) ** 2)
            scalars[:, :, s] = 1.0e-3 * np.exp(-(d / 0.5) ** 2)[:, None] * prof[None, :]

    out = dict(m)
    out.update(
        nVertLevels=K, num_scalars=ns, config=cfg,
        zgrid=zgrid, zz=zz, zxu=zxu, rdzw=vg["rdzw"], rdzu=vg["rdzu"], fzm=fzm, fzp=fzp,
        cf1=vg["cf1"], cf2=vg["cf2"], cf3=vg["cf3"],
        fEdge=fEdge, fVertex=fVertex, deriv_two=d2, zb=zb, zb3=zb3,
        # state (time level 1) and diag inputs of atm_init_coupled_diagnostics
        u=u, w=w, theta=theta, rho=rho, scalars=scalars, rho_base=rb, theta_base=tb,
    )
    return model_init(out, cfg)


def model_init_libm(m: dict, cfg: dict) -> dict:
    """The transcendental values of the model-init precompute, as the compiled reference gets them
    from the C library: meshDensity**0.25 per cell (atm_compute_damping_coefs 1113, mesh scaling 979)
    and per edge midpoint (meshScalingDel2, 963), and sin of the damping layer's argument per cell and
    level (1111; 0 where z <= config_zd).  model_init uses them, and mpas_dyc_model_init takes them
    (mesh.meshDensity_root4, meshDensityEdge_root4, dss_sin) so the device's precompute has the same
    bits."""
    zgrid, md = np.asarray(m["zgrid"]), np.asarray(m["meshDensity"])
    coe = np.asarray(m["cellsOnEdge"])
    zt_c = zgrid[:, m["nVertLevels"]]
    zmid = 0.5 * (zgrid[:, :-1] + zgrid[:, 1:])
    zd = cfg["config_zd"]
    arg = 0.5 * PII * (zmid - zd) / (zt_c[:, None] - zd)
    return {"meshDensity_root4": _pow(md, 0.25 * 1.0),
            "meshDensityEdge_root4": _pow((md[coe[:, 0]] + md[coe[:, 1]]) / 2.0, 0.25),
            "dss_sin": np.where(zmid > zd, np.sin(arg), 0.0)}


def model_init(out: dict, cfg: dict) -> dict:
    """The dycore's model-init precompute on the fields of an MPAS input stream
    (mpas_atm_core.F:311-463 and 927-1288): edge signs, zb_cell/zb3_cell, kiteForCell,
    adv_coefs compression and 3rd-order coupling, damping coefficients, mesh scaling,
    inverses, and -- when the input does not carry them -- defc_a/defc_b and
    coeffs_reconstruct.  ``out`` holds the mesh, zgrid, zb/zb3, deriv_two and the state;
    it is updated in place and returned."""
    m = out
    nC, nE, nV = m["nCells"], m["nEdges"], m["nVertices"]
    nz1 = m["nVertLevels"]
    nz = nz1 + 1
    coe, voe = m["cellsOnEdge"], m["verticesOnEdge"]
    c1, c2 = coe[:, 0], coe[:, 1]
    nEoC, eoc = m["nEdgesOnCell"], m["edgesOnCell"]
    zgrid, zb, zb3, d2 = m["zgrid"], m["zb"], m["zb3"], m["deriv_two"]
    coef3 = cfg["config_coef_3rd_order"]

    # ---- signs, zb_cell, kiteForCell (mpas_atm_core.F:987-1074)
    edgesOnCell_sign = np.zeros((nC, m["maxEdges"]))
    zb_cell = np.zeros((nC, m["maxEdges"], nz))
    zb3_cell = np.zeros((nC, m["maxEdges"], nz))
    kiteForCell = np.zeros((nC, m["maxEdges"]), dtype=np.int64)
    ac = np.arange(nC)
    for i in range(m["maxEdges"]):
        has = i < nEoC
        e = np.where(has, eoc[:, i], 0)
        first = coe[e, 0] == ac
        edgesOnCell_sign[:, i] = np.where(has, np.where(first, 1.0, -1.0), 0.0)
        side = np.where(first, 0, 1)
        zb_cell[:, i, :] = np.where(has[:, None], zb[e, side, :], 0.0)
        zb3_cell[:, i, :] = np.where(has[:, None], zb3[e, side, :], 0.0)
        v = np.where(has, m["verticesOnCell"][:, i], 0)
        kf = np.zeros(nC, dtype=np.int64)
        for j in range(2, -1, -1):
            kf = np.where(m["cellsOnVertex"][v, j] == ac, j, kf)
        kiteForCell[:, i] = np.where(has, kf, 0)          # 0-based (Fortran value - 1)
    eov = m["edgesOnVertex"]
    edgesOnVertex_sign = np.where(voe[eov, 1] == np.arange(nV)[:, None], 1.0, -1.0)

    # ---- adv_coefs compression and 3rd-order coupling (1121-1288)
    nAdv, advCells, adv_coefs, adv_coefs_3rd = adv_coef_compression(m, d2)
    adv_coefs_3rd = coef3 * adv_coefs_3rd
    zb3_cell = coef3 * zb3_cell
    if "defc_a" in m and "defc_b" in m:
        defc_a, defc_b = m["defc_a"], m["defc_b"]
    else:
        defc_a, defc_b = compute_defc(m)

    # damping (mpas_atm_core.F:1105-1116)
    lm = model_init_libm(m, cfg)
    zmid = 0.5 * (zgrid[:, :-1] + zgrid[:, 1:])
    zd, xnutr = cfg["config_zd"], cfg["config_xnutr"]
    sn = lm["dss_sin"]
    dss = np.where(zmid > zd, xnutr * (sn * sn), 0.0)
    dss = np.where(zmid > zd, dss / lm["meshDensity_root4"][:, None], 0.0)
    md = m["meshDensity"]
    if cfg["config_h_ScaleWithMesh"]:   # mesh scaling (927-984)
        msd2 = 1.0 / lm["meshDensityEdge_root4"]
        msd4 = 1.0 / _pow((md[c1] + md[c2]) / 2.0, 0.75)
    else:
        msd2 = np.ones(nE)
        msd4 = np.ones(nE)

    out.update(
        config=cfg, dss=dss, zb_cell=zb_cell, zb3_cell=zb3_cell,
        edgesOnCell_sign=edgesOnCell_sign, edgesOnVertex_sign=edgesOnVertex_sign, kiteForCell=kiteForCell,
        nAdvCellsForEdge=nAdv, advCellsForEdge=advCells, adv_coefs=adv_coefs, adv_coefs_3rd=adv_coefs_3rd,
        defc_a=defc_a, defc_b=defc_b, meshScalingDel2=msd2, meshScalingDel4=msd4,
        invAreaCell=1.0 / m["areaCell"], invDvEdge=1.0 / m["dvEdge"], invDcEdge=1.0 / m["dcEdge"],
        invAreaTriangle=1.0 / m["areaTriangle"],
    )
    # model-init precompute of the velocity reconstruction (mpas_atm_core.F:408-409)
    if "coeffs_reconstruct" not in out:
        out["coeffs_reconstruct"] = init_reconstruct(out)
    return out


def _jw_columns(lat, zgrid, zz, vg, R, moist):
    """JW columns for a chunk of cells (mpas_init_atm_cases.F:841-950); arrays (K, nc)."""
    nz1 = zz.shape[1]
    u0, t0b, t0, delta_t, dtdz, eta_t = 35.0, 250.0, 288.0, 4.8e5, 0.005, 0.2
    znut = eta_t
    zzT = np.ascontiguousarray(zz.T)
    ztemp = np.ascontiguousarray(0.5 * (zgrid[:, 1:] + zgrid[:, :-1]).T)
    ppb = P0 * _exp(-GRAVITY * ztemp / (RGAS * t0b))
    pb = _pow(ppb / P0, RGAS / CP)
    rb = ppb / (RGAS * t0b * zzT)
    tb = t0b / pb
    pp = np.zeros_like(ppb)
    rr = np.zeros_like(ppb)
    qv = np.zeros_like(ppb)
    phi = lat[None, :]
    dzw, dzu, fzp, fzm = vg["dzw"], vg["dzu"], vg["fzp"], vg["fzm"]
    sp, cp = _sincos(phi)  # one sincos(phi) per column (875-881)
    geo = ((-2.0 * _ipow(sp, 6) * (cp ** 2 + 1.0 / 3.0) + 10.0 / 63.0),
           (1.6 * _ipow(cp, 3) * (sp ** 2 + 2.0 / 3.0) - PII / 4.0) * R * OMEGA)
    for _ in range(10):
        eta = (ppb + pp) / P0
        etav = (eta - 0.252) * PII / 2.0
        dlt = znut - eta
        teta = t0 * _pow(eta, RGAS * dtdz / GRAVITY) + np.where(eta >= znut, 0.0, delta_t * (dlt * dlt * dlt * dlt * dlt))
        se, ce = _sincos(etav)  # sin(etav(k)) and cos(etav(k)) of one statement: one sincos
        temperature = teta + 0.75 * eta * PII * u0 / RGAS * se * np.sqrt(ce) * (
            geo[0] * 2.0 * u0 * _pow(ce, 1.5) + geo[1]) / (1.0 + 0.61 * qv)
        if moist:
            ptemp = ppb + pp
            relhum = np.where(ptemp < 50000.0, 0.0, np.where(ptemp > P0, 1.0, 1.0 - (np.maximum(P0 - ptemp, 0.0) / 50000.0) ** 1.25))
            relhum = np.minimum(0.40, relhum)
            es = np.where(temperature > 273.15,
                          1000.0 * 0.6112 * np.exp(17.67 * (temperature - 273.15) / (temperature - 29.65)),
                          1000.0 * 0.6112 * np.exp(21.8745584 * (temperature - 273.15) / (temperature - 7.66)))
            qsat = (287.04 / 461.6) * es / (ptemp - es)
            qsat = np.where(relhum == 0.0, 0.0, qsat)
            qv = relhum * qsat
        tt = temperature * (1.0 + 1.61 * qv)
        rzz = RGAS * zzT
        rbt = rb * (tt - t0b)
        for _ in range(25):
            rr = (pp / rzz - rbt) / tt
            ppi = np.empty_like(pp)
            ppi[0] = P0 - 0.5 * dzw[0] * GRAVITY * (1.25 * (rr[0] + rb[0]) * (1.0 + qv[0])
                                                    - 0.25 * (rr[1] + rb[1]) * (1.0 + qv[1]))
            ppi[0] -= ppb[0]
            term = rr + (rr + rb) * qv
            for k in range(nz1 - 1):
                ppi[k + 1] = ppi[k] - dzu[k + 1] * GRAVITY * (term[k] * fzp[k + 1] + term[k + 1] * fzm[k + 1])
            pp = 0.2 * ppi + 0.8 * pp
    p = _pow((ppb + pp) / P0, RGAS / CP)
    t = tt / p
    return ppb, pp, rb, rr, tb, t, qv


NLAT = 721  # mpas_init_atm_cases.F:441


def _jw_flux_zonal(lat1_in, lat2_in, dvEdge, R, vg, moist):
    """The rebalanced JW zonal flux of every edge, (nE, K): the JW state on the 721-point
    latitude grid (720-838), init_atm_recompute_geostrophic_wind (1215-1312), then
    init_atm_calc_flux_zonal per edge (1162-1213): the integral of u_2d over the edge's latitude
    span, linear interpolation in each latitude interval, summed in latitude order."""
    u0 = 35.0
    nz1 = vg["rdzw"].shape[0]
    dlat = 0.5 * PII / float(NLAT - 1)
    lat_2d = np.arange(NLAT, dtype=np.float64) * dlat
    hx = _jw_hx(lat_2d, R)
    zgrid = (1.0 - vg["ah"])[None, :] * (vg["sh"][None, :] * (vg["zt"] - hx[:, None]) + hx[:, None]) \
        + vg["ah"][None, :] * vg["sh"][None, :] * vg["zt"]                              # (nlat, K+1)
    zz = (vg["zw"][1:] - vg["zw"][:-1])[None, :] / (zgrid[:, 1:] - zgrid[:, :-1])
    # the 2-D columns never carry moisture (qv_2d stays 0 with the reference's moisture = .false.)
    ppb, pp, rb, rr, tb, t, qv = _jw_columns(lat_2d, zgrid, zz, vg, R, False)            # (K, nlat)
    rho_2d = rr + rb
    etavs_2d = ((ppb + pp) / P0 - 0.252) * PII / 2.0
    u_2d = u0 * (np.sin(2.0 * lat_2d) ** 2)[None, :] * _pow(np.cos(etavs_2d), 1.5)
    # init_atm_recompute_geostrophic_wind (1215-1312)
    zx = ((zgrid[1:, :] - zgrid[:-1, :]) / (dlat * R)).T                               # (K+1, nlat-1)
    rdx = 1.0 / (dlat * R)
    zzT = zz.T
    pgrad = rdx * (pp[:, 1:] / zzT[:, 1:] - pp[:, :-1] / zzT[:, :-1])
    fzm, fzp, rdzw = vg["fzm"], vg["fzp"], vg["rdzw"]
    dpzx = np.zeros((nz1 + 1, NLAT - 1))
    dpzx[0] = .5 * zx[0] * (vg["cf1"] * (pp[0, 1:] + pp[0, :-1]) + vg["cf2"] * (pp[1, 1:] + pp[1, :-1])
                            + vg["cf3"] * (pp[2, 1:] + pp[2, :-1]))
    for k in range(1, nz1):
        dpzx[k] = .5 * zx[k] * (fzm[k] * (pp[k, 1:] + pp[k, :-1]) + fzp[k] * (pp[k - 1, 1:] + pp[k - 1, :-1]))
    pgrad = pgrad - rdzw[:, None] * (dpzx[1:] - dpzx[:-1])
    u = .5 * (u_2d[:, :-1] + u_2d[:, 1:])
    ru = u * (rho_2d[:, :-1] + rho_2d[:, 1:]) * .5
    phi = (lat_2d[:-1] + lat_2d[1:]) / 2.0
    f = 2.0 * OMEGA * np.sin(phi)
    qtot = .5 * (qv[:, :-1] + qv[:, 1:])
    for _ in range(50):
        ru = np.where(f == 0.0, 0.0,
                      -(1.0 / (1.0 + qtot) * pgrad + (_tan(phi) / R)[None, :] * u * ru) / np.where(f == 0.0, 1.0, f))
        u = ru * 2.0 / (rho_2d[:, :-1] + rho_2d[:, 1:])
    u_2d = u_2d.copy()
    u_2d[:, 1:-1] = (ru[:, :-1] + ru[:, 1:]) * .5
    u_2d[:, 0] = (3.0 * u_2d[:, 1] - u_2d[:, 2]) * .5
    u_2d[:, -1] = (3.0 * u_2d[:, -2] - u_2d[:, -3]) * .5
    # init_atm_calc_flux_zonal (1162-1213), all edges at once: the latitude intervals i each edge
    # overlaps, in ascending order
    a1, a2 = np.abs(lat1_in), np.abs(lat2_in)
    lo = np.where(a2 <= a1, a2, a1)
    hi = np.where(a2 <= a1, a1, a2)
    i0 = np.maximum(np.floor(lo / dlat).astype(np.int64) - 1, 0)
    i1 = np.minimum(np.ceil(hi / dlat).astype(np.int64) + 1, NLAT - 2)
    acc = np.zeros((lo.shape[0], nz1))
    dl_last = np.zeros(lo.shape[0])
    u_2dT = np.ascontiguousarray(u_2d.T)  # (nlat, K)
    for e0 in range(0, lo.shape[0], 32768):  # edge batches that stay in cache
        s_ = slice(e0, min(lo.shape[0], e0 + 32768))
        lo_, hi_, i0_, i1_ = lo[s_], hi[s_], i0[s_], i1[s_]
        ac = np.zeros((lo_.shape[0], nz1))
        dll = np.zeros(lo_.shape[0])
        for j in range(int((i1_ - i0_).max()) + 1):
            i = np.minimum(i0_ + j, NLAT - 2)
            ok = (i0_ + j <= i1_) & (lo_ <= lat_2d[i + 1]) & (hi_ >= lat_2d[i])
            dl = lat_2d[i + 1] - lat_2d[i]
            da = (np.maximum(lo_, lat_2d[i]) - lat_2d[i]) / dl
            db = (np.minimum(hi_, lat_2d[i + 1]) - lat_2d[i]) / dl
            w1 = (db - da) - 0.5 * (db - da) ** 2
            w2 = 0.5 * (db - da) ** 2
            ac = np.where(ok[:, None], ac + w1[:, None] * u_2dT[i] + w2[:, None] * u_2dT[i + 1], ac)
            dll = np.where(ok, dl, dll)
        acc[s_] = ac
        dl_last[s_] = dll
    sgn = np.copysign(1.0, lat2_in - lat1_in)
    # the reference scales by its loop variable dlat: the width of the last interval it summed
    return sgn[:, None] * acc * dl_last[:, None] * R / dvEdge[:, None] / u0
