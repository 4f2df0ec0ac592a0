"""C-ABI boundary checks that run without a GPU: libdcp.so loads, exports every
symbol include/dcp.h declares, and refuses to compute without a device (there
is no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

import dcp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "dcp.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dcp_[A-Za-z_0-9]+)\s*\(", text)))


def test_header_matches_binding_list():
    assert declared_symbols() == sorted(dcp.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(dcp.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_abi_version_matches_header():
    """DCP_ABI_VERSION in include/dcp.h, the library's dcp_abi_version() and the
    binding's ABI_VERSION agree; the binding refuses a library built against
    another header (layout changes such as [n][27][3] -> [n][64][3] geometry)."""
    text = open(os.path.join(ROOT, "include", "dcp.h")).read()
    v = int(re.search(r"#define DCP_ABI_VERSION (\d+)", text).group(1))
    pts = int(re.search(r"#define DCP_CELL_SUPPORT_POINTS (\d+)", text).group(1))
    assert v == dcp.ABI_VERSION == ctypes.CDLL(dcp.LIB_PATH).dcp_abi_version()
    assert pts == dcp.CELL_SUPPORT_POINTS == dcp.HostMesh(refine=0).cell_geometry.shape[1]


def test_no_cpu_fallback():
    if dcp.lib().dcp_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(dcp.DcpError) as e:
        dcp.Context()
    assert e.value.code == dcp.DCP_ERR_DEVICE


def test_host_mesh_helpers_without_gpu():
    m = dcp.HostMesh(refine=1)
    assert m.cell_geometry.shape == (48, 64, 3)  # MappingQ(3) support points
    assert m.cell_nse_dofs.shape == (48, 89)


@pytest.mark.parametrize("r", [0, 1, 2, 3, 4])
def test_upload_conversion_shell(r):
    m = dcp.HostMesh(refine=r)
    ncol = m.check()
    # refine >= 1: the structured shell colouring (layer parity x a lateral
    # 4-colouring of the cubed-sphere patches, checked on every vertex-sharing
    # pair inside the library) replaces the greedy one's 14 classes
    assert ncol == 8 if r > 0 else 2 <= ncol <= 8


@pytest.mark.parametrize("r", [1, 2, 3])
def test_upload_accepts_periodic_cube(r):
    """BASELINE C2: the periodic x/y identities of the cuboid
    (make_periodicity_constraints, boussinesq_model.tpp:265-285) are folded into
    the cell maps at upload (host-only dry run)."""
    m = dcp.HostMesh(cuboid=True, refine=r)
    assert 8 <= m.check() <= 64


def test_upload_rejects_partly_periodic_node():
    m = dcp.HostMesh(cuboid=True, refine=1)
    nc = m.nse_constraints
    # turn one periodic identity line into a coupling to two nodes
    lens = np.diff(nc.entry_ptr)
    l = int(np.flatnonzero((lens == 1) & (nc.line_dof < m.n_u))[0])
    e = nc.entry_ptr[l]
    w = nc.entry_w.copy()
    w[e] = 0.5
    bad = dcp.ConstraintSet(nc.line_dof, nc.entry_ptr, nc.entry_dof, w, nc.inhomogeneity)
    with pytest.raises(dcp.DcpError) as err:
        m.check(nse_constraints=bad)
    assert err.value.code == dcp.DCP_ERR_UNSUPPORTED


def test_upload_rejects_bad_dof_layout():
    m = dcp.HostMesh(refine=1)
    m.cell_nse_dofs = m.cell_nse_dofs.copy()
    m.cell_nse_dofs[0, 0], m.cell_nse_dofs[0, 1] = m.cell_nse_dofs[0, 1], m.cell_nse_dofs[0, 0]
    with pytest.raises(dcp.DcpError):
        m.check()


@pytest.mark.parametrize("r", [1, 2, 3])
@pytest.mark.parametrize("all_cells", [False, True])
def test_separable_geometry_detection(r, all_cells):
    """The shell's MappingQ(3) support points are rho_c * Phi_ab: one 2D table
    per column of cells (6 N^2; twice that with deal.II 9.2's trilinear
    interior cells, whose Phi is the bilinear blend) and one radial table per
    layer (N)."""
    m = dcp.HostMesh(refine=r, mapping_q_on_all_cells=all_cells)
    N = 2 ** r
    kinds = 1 if (all_cells or N <= 2) else 2
    assert m.geometry_info() == (True, kinds * 6 * N * N, N)
    # a smooth displacement breaks the separability: general streamed path
    m.cell_geometry = m.cell_geometry.copy()
    X = m.cell_geometry.reshape(-1, 3)
    X += 0.02 * np.sin(3.0 * X[:, [1, 2, 0]]) * np.cos(2.0 * X[:, [2, 0, 1]])
    assert m.geometry_info() == (False, 0, 0)
