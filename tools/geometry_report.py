"""Quantifies the geometry change of round 2:
(a) vertex displacement of SphericalManifold refinement (deal.II's rule)
    against the equiangular cube-sphere round 1 used, per refinement;
(b) element matrices of MappingQ(3) against a Q2 isoparametric map through the
    same Q2 support points, on boundary (cubic) cells.
usage: python tools/geometry_report.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "3d-dycoreplanet_amd"), os.path.join(HERE, "..", "oracle")]
import numpy as np  # noqa: E402
import dcp  # noqa: E402
import oracle_py  # noqa: E402

GL = np.array([0.0, 0.5 - 0.5 / np.sqrt(5.0), 0.5 + 0.5 / np.sqrt(5.0), 1.0])
VTX = [0, 3, 12, 15, 48, 51, 60, 63]


def lag2(a, x):
    return [2 * (x - 0.5) * (x - 1), -4 * x * (x - 1), 2 * x * (x - 0.5)][a]


for r in (1, 2, 3, 4, 5):
    m = dcp.HostMesh(refine=r)
    N = 2 ** r
    V = m.cell_geometry[:, VTX].reshape(-1, 3)
    d = V / np.linalg.norm(V, axis=1)[:, None]
    worst = 0.0
    for v in d:
        ax = int(np.argmax(np.abs(v)))
        t = [k for k in range(3) if k != ax]
        a = np.arctan(v[t] / abs(v[ax])) / (np.pi / 4)      # in [-1, 1]
        s = np.round((a + 1) * N / 2) * 2 / N - 1           # nearest lattice line
        e = np.zeros(3)
        e[ax] = np.sign(v[ax])
        e[t] = np.tan(np.pi / 4 * s)
        e /= np.linalg.norm(e)
        worst = max(worst, np.arccos(np.clip(e @ v, -1, 1)))
    h = (np.pi / 2) / N
    line = "r=%d  max vertex angle equiangular vs SphericalManifold: %.3e rad = %.3f cell widths" % (
        r, worst, worst / h)
    if r <= 3:
        ph = dcp.classic_physics()
        u = np.zeros(m.n_u + m.n_p)
        devs = []
        for c in range(0, m.n_cells, max(1, m.n_cells // 24)):
            X3 = m.cell_geometry[c]
            rad = np.linalg.norm(X3[VTX], axis=1)
            if not (np.isclose(rad.min(), 1.0) or np.isclose(rad.max(), 3.0)):
                continue
            # Q2 nodes = the cubic map at (a, b, c) / 2; their Q2 interpolant at the GL points
            n2 = m.node_xyz[m.cell_nse_dofs[c, [4 * v for v in range(8)] + list(range(32, 89, 3))] // 3]
            # lexicographic Q2 node positions from the FESystem order (vertices, lines, faces, interior)
            H2L = [0, 2, 6, 8, 18, 20, 24, 26, 3, 5, 1, 7, 21, 23, 19, 25, 9, 11, 15, 17, 12, 14, 10,
                   16, 4, 22, 13]
            P = np.zeros((27, 3))
            P[H2L] = n2
            X2 = np.zeros((64, 3))
            for t in range(64):
                x = (GL[t % 4], GL[(t // 4) % 4], GL[t // 16])
                for n in range(27):
                    X2[t] += lag2(n % 3, x[0]) * lag2((n // 3) % 3, x[1]) * lag2(n // 9, x[2]) * P[n]
            K3, _ = oracle_py.cell_nse_system(ph, X3, u[m.cell_nse_dofs[c]], m.T0[m.cell_T_dofs[c]])
            K2, _ = oracle_py.cell_nse_system(ph, X2, u[m.cell_nse_dofs[c]], m.T0[m.cell_T_dofs[c]])
            devs.append(np.max(np.abs(K3 - K2)) / np.max(np.abs(K3)))
        line += "; boundary-cell element matrix MappingQ(3) vs Q2-iso: max rel %.2e" % max(devs)
    print(line, flush=True)
