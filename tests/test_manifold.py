"""deal.II geometry rules of the host setup (csrc/manifold.cpp) against an
independent numpy restatement: SphericalManifold's get_new_points (weighted
spherical average: the linear guess when the points are within 2e-2 squared
chord of each other, otherwise the minimiser of sum_i w_i theta_i^2) for the
MappingQ(3) support points (boussinesq_model.tpp:20), and the hyper_shell
refinement rule (line midpoints = geodesic midpoints, quad centres from
TriaAccessor::center(true, true)'s weights). Parity with deal.II itself is
unpinned (not in this image); this pins the restatement to the published
formulas."""
import numpy as np
import pytest

import dcp

GL = np.array([0.0, 0.5 - 0.5 / np.sqrt(5.0), 0.5 + 0.5 / np.sqrt(5.0), 1.0])
VTX = [0, 3, 12, 15, 48, 51, 60, 63]  # lexicographic support points of the 8 vertices


def spherical_mean(dirs, w, x):
    """Fixed point x <- exp_x(sum_i w_i log_x(d_i)) on the unit sphere (the
    stationary point of sum_i w_i theta_i^2 for weights summing to 1)."""
    for _ in range(100):
        v = np.zeros(3)
        for d, wi in zip(dirs, w):
            c = np.clip(d @ x, -1, 1)
            t = d - c * x
            s = np.linalg.norm(t)
            if s > 1e-300:
                v += wi * np.arctan2(s, c) * t / s
        th = np.linalg.norm(v)
        if th < 1e-16:
            break
        x = np.cos(th) * x + np.sin(th) * v / th
    return x


def new_point(src, w):
    r = np.linalg.norm(src, axis=1)
    dirs = src / r[:, None]
    rho = w @ r
    g = w @ dirs
    g /= np.linalg.norm(g)
    dmax = max(np.sum((dirs[i] - dirs[k]) ** 2) for i in range(len(dirs)) for k in range(i))
    return rho * (g if dmax < 2e-2 else spherical_mean(dirs, w, g))


def trilinear_weights(x, y, z):
    return np.array([((1 - x) if v & 1 == 0 else x) * ((1 - y) if v & 2 == 0 else y) *
                     ((1 - z) if v & 4 == 0 else z) for v in range(8)])


@pytest.mark.parametrize("r", [1, 2, 4])
@pytest.mark.parametrize("all_cells", [False, True])
def test_mapping_support_points(r, all_cells):
    m = dcp.HostMesh(refine=r, mapping_q_on_all_cells=all_cells)
    N = 2 ** r
    rng = np.random.default_rng(7)
    cells = rng.choice(m.n_cells, size=min(m.n_cells, 24), replace=False)
    worst = 0.0
    for c in cells:
        X = m.cell_geometry[c]
        V = X[VTX]
        rad = np.linalg.norm(V, axis=1)
        boundary = np.isclose(rad.min(), 1.0) or np.isclose(rad.max(), 3.0)
        for t in range(64):
            w = trilinear_weights(GL[t % 4], GL[(t // 4) % 4], GL[t // 16])
            ref = new_point(V, w) if (all_cells or boundary) else w @ V
            worst = max(worst, np.max(np.abs(ref - X[t])))
    assert worst < 1e-13, worst


def test_refinement_rule_r1():
    """r = 1: line midpoints of the coarse cube-sphere are geodesic midpoints
    and the panel centres are (+-1, 0, 0) etc. (symmetric quad rule)."""
    m = dcp.HostMesh(refine=1)
    V = m.cell_geometry[:, VTX].reshape(-1, 3)
    dirs = np.unique(np.round(V / np.linalg.norm(V, axis=1)[:, None], 12), axis=0)
    s3, s2 = 1 / np.sqrt(3), 1 / np.sqrt(2)
    expect = set()
    for a in (-1, 1):
        for b in (-1, 1):
            for c in (-1, 1):
                expect.add((a * s3, b * s3, c * s3))
    for ax in range(3):
        for sgn in (-1, 1):
            e = [0.0, 0.0, 0.0]
            e[ax] = sgn
            expect.add(tuple(e))
            for ax2 in range(3):
                if ax2 == ax:
                    continue
                for sgn2 in (-1, 1):
                    e2 = [0.0, 0.0, 0.0]
                    e2[ax] = sgn * s2
                    e2[ax2] = sgn2 * s2
                    expect.add(tuple(e2))
    expect = np.unique(np.round(np.array(sorted(expect)), 12), axis=0)
    assert dirs.shape == expect.shape and np.allclose(dirs, expect, atol=1e-12)


def test_refinement_rule_r2_quad_centres():
    """r = 2: the centre vertex of every level-1 spherical quad is
    get_new_point(4 corners (-1/4), 4 geodesic line midpoints (+1/2))."""
    m1 = dcp.HostMesh(refine=1)
    m2 = dcp.HostMesh(refine=2)
    V2 = m2.cell_geometry[:, VTX].reshape(-1, 3)
    U2 = V2 / np.linalg.norm(V2, axis=1)[:, None]
    checked = 0
    for c in range(m1.n_cells):
        V = m1.cell_geometry[c][VTX]
        r = np.linalg.norm(V, axis=1)
        if not np.isclose(r.min(), 1.0):
            continue
        q = V[:4] / r[:4, None]  # inner face corners (local z = 0)
        def mid(a, b):
            s = q[a] + q[b]
            return s / np.linalg.norm(s)
        lines = [mid(0, 2), mid(1, 3), mid(0, 1), mid(2, 3)]
        src = np.vstack([q, lines])
        w = np.array([-0.25] * 4 + [0.5] * 4)
        ctr = new_point(src, w)
        assert np.min(np.linalg.norm(U2 - ctr, axis=1)) < 1e-13
        checked += 1
    assert checked == 24
