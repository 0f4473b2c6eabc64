"""The float certification of mesh_to_spc's per-parent level kernel (csrc/spc.hip, m2s_children)
restated in numpy float32 and checked against a float64 restatement of the reference's
TriangleVoxelSAT (mesh_to_spc_cuda.cu:96-159, as tri_voxel_test): every child decision the margins
certify (pass or reject) must be the reference's, on random, plane-through-corner, tiny,
sliver and voxel-plane-aligned triangles at levels 1..12.  (A check of the margin argument in the
kernel's comment, not of the kernel: the GPU tests compare the kernel's octrees with the oracle.)"""
import numpy as np
f32 = np.float32

def ref_test(fa, fb, fc, c, h):
    # tri_voxel_test: v = (double)(f - c) in float; unit edges in double; 13 axes
    va = (fa - c).astype(np.float64); vb = (fb - c).astype(np.float64); vc = (fc - c).astype(np.float64)
    def dnorm(x):
        with np.errstate(all='ignore'):
            inv = 1.0 / np.sqrt((x * x).sum(-1, keepdims=True))
            return inv * x
    ab, bc, ca = dnorm(vb - va), dnorm(vc - vb), dnorm(va - vc)
    z = np.zeros_like(ab[..., 0]); o = np.ones_like(z)
    axes = []
    for e in (ab, bc, ca): axes.append(np.stack([z, -e[..., 2], e[..., 1]], -1))
    for e in (ab, bc, ca): axes.append(np.stack([e[..., 2], z, -e[..., 0]], -1))
    for e in (ab, bc, ca): axes.append(np.stack([-e[..., 1], e[..., 0], z], -1))
    axes += [np.stack([o, z, z], -1), np.stack([z, o, z], -1), np.stack([z, z, o], -1)]
    n = np.cross(ab, bc); axes.append(n)
    ok = np.ones(z.shape, bool)
    hd = h.astype(np.float64)
    with np.errstate(all='ignore'):
        for a in axes:
            # ddot = a.x*b.x + a.y*b.y + a.z*b.z left to right
            d = np.stack([(v[..., 0] * a[..., 0] + v[..., 1] * a[..., 1]) + v[..., 2] * a[..., 2] for v in (va, vb, vc)], -1)
            mx = np.max(d, -1); mn = np.min(d, -1)
            r = hd * ((np.abs(a[..., 0]) + np.abs(a[..., 1])) + np.abs(a[..., 2]))
            fr = r.astype(np.float32)
            # NaN in fmax: C fmax ignores NaN operands; np.maximum propagates. emulate fmax
            fdv = np.where(np.isnan(-mx), mn, np.where(np.isnan(mn), -mx, np.maximum(-mx, mn))).astype(np.float32)
            ok &= fdv <= fr
    return ok

def children(v, px, py, pz, level):
    # float32 emulation of m2s_children's certification: returns (pass_cert, rej_cert, amb) 8-bit per row
    vs = f32(2.0) / f32(2 ** level); h = f32(0.5 * vs)
    C = np.stack([(f32(2) * p.astype(f32)) * vs + (h - f32(1)) + h for p in (px, py, pz)], -1).astype(f32)
    fa, fb, fc = v[:, 0], v[:, 1], v[:, 2]
    w = [(fa - C).astype(f32), (fb - C).astype(f32), (fc - C).astype(f32)]
    E = [(fb - fa).astype(f32), (fc - fb).astype(f32), (fa - fc).astype(f32)]
    V = np.max(np.abs(np.stack(w, 1)).reshape(len(v), -1), 1)
    Em = np.max(np.abs(np.stack(E, 1)).reshape(len(v), -1), 1)
    U = (V + f32(2) * h + Em).astype(f32)
    N = len(v)
    rej = np.zeros((N, 8), bool); amb = np.zeros((N, 8), bool)
    cb = np.array([[(c >> 2) & 1, (c >> 1) & 1, c & 1] for c in range(8)])
    # box axes exact
    for q in range(3):
        for b in (0, 1):
            c = (C[:, q] + h) if b else (C[:, q] - h)
            u = np.stack([(v[:, k, q] - c).astype(f32) for k in range(3)], -1)
            fd = np.maximum(-u.max(-1), u.min(-1))
            bad = ~(fd <= h)
            rej[:, cb[:, q] == b] |= bad[:, None]
    Me = (f32(1 / 131072) * U * U).astype(f32)
    def axis(P, a, M):
        pmax = P.max(-1); pmin = P.min(-1)
        R = (h * ((np.abs(a[:, 0]) + np.abs(a[:, 1])) + np.abs(a[:, 2]))).astype(f32)
        for c in range(8):
            sg = np.where(cb[c] == 1, f32(1), f32(-1)).astype(f32)
            sv = ((sg[0] * (h * a[:, 0])) + (sg[1] * (h * a[:, 1]))) + (sg[2] * (h * a[:, 2]))
            S = (np.maximum(sv - pmax, pmin - sv) - R).astype(f32)
            rej[:, c] |= S > M
            amb[:, c] |= ~(S < -M) & ~(S > M)
    z = np.zeros(N, f32)
    for e in E:
        for a in (np.stack([z, -e[:, 2], e[:, 1]], -1), np.stack([e[:, 2], z, -e[:, 0]], -1), np.stack([-e[:, 1], e[:, 0], z], -1)):
            a = a.astype(f32)
            P = np.stack([((wk[:, 0] * a[:, 0]) + (wk[:, 1] * a[:, 1])) + wk[:, 2] * a[:, 2] for wk in w], -1).astype(f32)
            axis(P, a, Me)
    n = np.stack([E[0][:, 1] * E[1][:, 2] - E[0][:, 2] * E[1][:, 1], E[0][:, 2] * E[1][:, 0] - E[0][:, 0] * E[1][:, 2],
                  E[0][:, 0] * E[1][:, 1] - E[0][:, 1] * E[1][:, 0]], -1).astype(f32)
    P = np.stack([((wk[:, 0] * n[:, 0]) + (wk[:, 1] * n[:, 1])) + wk[:, 2] * n[:, 2] for wk in w], -1).astype(f32)
    axis(P, n, (f32(1 / 32768) * U * U * (Em + f32(1 / 1024) * U)).astype(f32))
    bad = ~(U < f32(1e12))
    amb[bad] = True; rej[bad] = False
    return rej, amb, h, cb



def test_children_certification_matches_reference():
    rng = np.random.default_rng(0)
    tot = cert = 0
    for level in (1, 3, 5, 7, 9, 12):
        n = 2 ** level
        for kind in ('rand', 'plane', 'tiny', 'sliver', 'grid', 'small', 'smallplane'):
            M = 3000
            P = rng.integers(0, n // 2 if level > 0 else 1, (M, 3))
            vsz = 2.0 / (n // 2)
            Cc = -1 + (P + 0.5) * vsz
            if kind == 'rand':
                v = Cc[:, None, :] + rng.normal(0, vsz, (M, 3, 3))
            elif kind == 'plane':  # plane through parent centre / child corners
                a = rng.normal(size=(M, 3)); a /= np.linalg.norm(a, axis=1, keepdims=True)
                t1 = np.cross(a, rng.normal(size=(M, 3))); t2 = np.cross(a, t1)
                coef = rng.uniform(-2, 2, (M, 3, 2)) * vsz
                off = rng.choice([0.0, 0.5, 1.0], (M, 1)) * vsz * (rng.integers(0, 2, (M, 1)) * 2 - 1)
                v = Cc[:, None, :] + coef[..., :1] * t1[:, None] + coef[..., 1:] * t2[:, None] + (off * a)[:, None]
            elif kind == 'tiny':
                corner = Cc + rng.choice([-0.5, 0, 0.5], (M, 3)) * vsz
                v = corner[:, None, :] + rng.normal(0, 1e-7, (M, 3, 3))
            elif kind == 'sliver':
                a0 = Cc + rng.uniform(-1, 1, (M, 3)) * vsz; d = rng.normal(0, vsz, (M, 3))
                v = np.stack([a0, a0 + d, a0 + d * rng.uniform(0, 1, (M, 1)) + rng.normal(0, 1e-8, (M, 3))], 1)
            elif kind in ('small', 'smallplane'):  # edges ~1/100 of a level-2 voxel (cfg4's first levels)
                at = 0.5 * rng.choice([-1.0, 0.0, 1.0], (M, 3)) if kind == 'smallplane' else rng.uniform(-0.6, 0.6, (M, 3))
                es = 0.01 * rng.choice([1.0, 1e-2, 1e-4], (M, 1, 1))
                v = (Cc + at * vsz + rng.normal(0, 0.01, (M, 3)) * (kind == 'smallplane'))[:, None, :] + \
                    rng.normal(0, 1, (M, 3, 3)) * es
            else:  # axis aligned on child planes
                k = rng.integers(0, 3, M)
                base = Cc + rng.choice([-0.5, 0, 0.5], (M, 3)) * vsz
                v = base[:, None, :] + rng.uniform(-1, 1, (M, 3, 3)) * vsz
                v[np.arange(M), :, k] = base[np.arange(M), k][:, None]
            v = v.astype(f32)
            rej, amb, h, cb = children(v, P[:, 0], P[:, 1], P[:, 2], level)
            for c in range(8):
                # the child's centre as voxel_center computes it: fmaf(px_c, vs, h - 1) (exact)
                vs = f32(2.0) / f32(2 ** level)
                cc = np.stack([((2 * P[:, q] + cb[c][q]).astype(f32) * vs + (h - f32(1))).astype(f32) for q in range(3)], -1)
                ok = ref_test(v[:, 0], v[:, 1], v[:, 2], cc, np.full(M, h, f32))
                certp = ~rej[:, c] & ~amb[:, c]
                certr = rej[:, c]
                assert not np.any(certp & ~ok), (level, kind, c, np.flatnonzero(certp & ~ok)[:5])
                assert not np.any(certr & ok), (level, kind, c, np.flatnonzero(certr & ok)[:5])
                tot += M; cert += int((certp | certr).sum())
    assert cert / tot > 0.8  # most children decided without the full test
