"""ctypes binding of libdcp.so (include/dcp.h) — the host-side view of the
MI355X Boussinesq hot path, mirroring the reference model's member calls
(include/core/boussinesq_model.tpp):

    assemble_nse_system      -> Context.assemble_nse_system()
    build_nse_preconditioner -> Context.build_nse_preconditioner()
    assemble_temperature_*   -> Context.assemble_temperature_matrix()/_rhs()
    solve_NSE_block_...      -> Context.solve_nse()
    solve_temperature        -> Context.solve_temperature()

There is no CPU fallback: loading fails loudly when libdcp.so is missing and
every compute call raises DcpError when no GPU is present.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DCP_LIBRARY: another build of the same sources (tools/ probes of compile-time variants)
LIB_PATH = os.environ.get("DCP_LIBRARY") or os.path.join(_HERE, "libdcp.so")

DCP_OK, DCP_NOT_CONVERGED = 0, 1
DCP_ERR_INVALID, DCP_ERR_UNSUPPORTED, DCP_ERR_DEVICE, DCP_ERR_STATE = -1, -2, -3, -4
NSE_SOLUTION, OLD_NSE_SOLUTION, T_SOLUTION, OLD_T_SOLUTION, NSE_RHS, T_RHS = range(6)
ASSEMBLE_MATRIX, ASSEMBLE_RHS = 1, 2
OPT_SCHUR_EXPLICIT = 1
OPT_FEEC_ZERO_MEAN = 2
OPT_MATRIX_FREE = 3
OPT_FUSED_CHAIN = 4
OPT_FGMRES_MAX_OUTER = 5
OPT_ASSEMBLE_VELOCITY_BLOCK = 6
OPT_ELEMENT_MFMA = 9
OPT_GRAM_SCHMIDT = 7
OPT_FEEC_FIXED_INNER = 8
OPT_LOG_HISTORY = 10
OPT_INNER_MAX_STEPS = 11
OPT_SCHUR_FIXED_INNER = 12
OPT_HANDOFF_SPIN_LIMIT = 13
OPT_BLOCK_FIXED_INNER = 14
OPT_MATRIX_POWERS = 15
OPT_FEEC_BLOCK_PRECONDITIONER = 16
OPT_T_FIXED_CG = 17
ABI_VERSION = 5            # include/dcp.h DCP_ABI_VERSION
CELL_SUPPORT_POINTS = 64   # include/dcp.h DCP_CELL_SUPPORT_POINTS

# Every symbol include/dcp.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "dcp_abi_version", "dcp_ctx_create", "dcp_ctx_destroy", "dcp_last_error", "dcp_device_count",
    "dcp_set_physics", "dcp_set_time_step", "dcp_set_option", "dcp_mesh_upload", "dcp_mesh_check", "dcp_state_set",
    "dcp_state_get", "dcp_state_copy", "dcp_state_device_ptr", "dcp_assemble_nse_system",
    "dcp_build_nse_preconditioner", "dcp_assemble_temperature_matrix",
    "dcp_assemble_temperature_rhs", "dcp_solve_nse", "dcp_solve_nse_schur", "dcp_solve_temperature",
    "dcp_max_velocity", "dcp_cfl_number", "dcp_advance_state", "dcp_nse_vmult", "dcp_velocity_vmult", "dcp_mesh_geometry_info", "dcp_run",
    "dcp_schur_vmult", "dcp_block_preconditioner_vmult", "dcp_nse_matrix_export",
    "dcp_T_matrix_export", "dcp_precond_diagonals", "dcp_cell_nse_system",
    "dcp_get_timings", "dcp_pattern_info", "dcp_host_mesh_create", "dcp_host_mesh_destroy",
    "dcp_host_mesh_renumber_cuthill_mckee",
    "dcp_host_mesh_renumber_dealii",
    "dcp_host_mesh_view_get", "dcp_host_mesh_initial_temperature", "dcp_prm_load",
    "dcp_nccl_unique_id", "dcp_group_create", "dcp_group_destroy", "dcp_partition_info",
    "dcp_feec_mesh_upload", "dcp_feec_assemble_nse_system", "dcp_feec_build_nse_preconditioner",
    "dcp_feec_solve_nse", "dcp_feec_cell_system", "dcp_feec_matrix_export",
    "dcp_host_feec_view_get", "dcp_schur_layout", "dcp_assembly_layout",
    "dcp_feec_partition_info",
    "dcp_mesh2d_partition_info", "dcp_time_operator",
    "dcp_write_vtu", "dcp_write_pvtu_record", "dcp_solver_history", "dcp_timer_summary",
    "dcp_timer_section", "dcp_timer_record", "dcp_timer_reset",
    "dcp_mesh2d_upload", "dcp_mesh2d_check", "dcp_host_mesh2d_create", "dcp_host_mesh2d_view_get",
    "dcp_mesh_upload_distributed", "dcp_dist_partition_info", "dcp_dist_partition_info_field",
    "dcp_partition_info_field", "dcp_state_set_owned",
    "dcp_state_get_owned", "dcp_scatter_info", "dcp_matrix_powers_info", "dcp_device_memory",
    "dcp_comm_info", "dcp_local_sizes",
    "dcp_nse_coupling_export",
    "dcp_halo_selftest", "dcp_allreduce_selftest", "dcp_write_feec_vtu", "dcp_write_feec_pvtu_record",
]


class DcpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"dcp error {code}: {msg}")
        self.code = code


class Physics(C.Structure):
    _fields_ = [
        ("time_step", C.c_double), ("one_over_reynolds", C.c_double),
        ("one_over_peclet", C.c_double), ("expansion_coefficient", C.c_double),
        ("temperature_ref", C.c_double), ("gravity_scale", C.c_double),
        ("gravity_constant", C.c_double), ("coriolis_scale", C.c_double),
        ("omega", C.c_double), ("cuboid", C.c_int), ("nse_solver_interval", C.c_int),
        ("temperature_degree", C.c_int),
    ]


class Constraints(C.Structure):
    _fields_ = [
        ("n_lines", C.c_int), ("line_dof", C.POINTER(C.c_int)),
        ("entry_ptr", C.POINTER(C.c_int)), ("entry_dof", C.POINTER(C.c_int)),
        ("entry_w", C.POINTER(C.c_double)), ("inhomogeneity", C.POINTER(C.c_double)),
    ]


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("rank", C.c_int), ("world_size", C.c_int),
                ("nccl_id", C.c_void_p), ("group", C.c_void_p)]


class Timings(C.Structure):
    _fields_ = [
        ("assemble_nse_ms", C.c_double), ("build_precond_ms", C.c_double),
        ("assemble_T_matrix_ms", C.c_double), ("assemble_T_rhs_ms", C.c_double),
        ("solve_nse_ms", C.c_double), ("solve_T_ms", C.c_double),
        ("schur_apply_ms_avg", C.c_double), ("schur_applies", C.c_long),
        ("stokes_apply_ms_avg", C.c_double), ("velocity_apply_ms_avg", C.c_double),
        ("stokes_applies", C.c_long), ("velocity_applies", C.c_long),
        ("a_solve_iterations", C.c_long), ("handoff_timeouts", C.c_long),
    ]


class MeshView(C.Structure):
    _fields_ = [
        ("n_cells", C.c_int), ("n_u", C.c_int), ("n_p", C.c_int), ("n_T", C.c_int),
        ("n_vnodes", C.c_int),
        ("cell_nse_dofs", C.POINTER(C.c_int32)), ("cell_T_dofs", C.POINTER(C.c_int32)),
        ("cell_geometry", C.POINTER(C.c_double)), ("cell_diameter", C.POINTER(C.c_double)),
        ("node_xyz", C.POINTER(C.c_double)), ("nse", Constraints), ("T", Constraints),
    ]


class FeecMeshView(C.Structure):
    _fields_ = [
        ("n_cells", C.c_int), ("n_w", C.c_int), ("n_u", C.c_int), ("n_p", C.c_int),
        ("n_T", C.c_int),
        ("cell_w", C.POINTER(C.c_int32)), ("sign_w", C.POINTER(C.c_int8)),
        ("cell_u", C.POINTER(C.c_int32)), ("sign_u", C.POINTER(C.c_int8)),
        ("cell_vertices", C.POINTER(C.c_double)), ("cell_diameter", C.POINTER(C.c_double)),
        ("cell_T_dofs", C.POINTER(C.c_int32)), ("w_fixed", C.POINTER(C.c_uint8)),
        ("u_fixed", C.POINTER(C.c_uint8)), ("T", Constraints),
    ]


class Mesh2DView(C.Structure):
    """dcp_mesh2d: the 2D model's DoFs, geometry and constraints."""
    _fields_ = [
        ("n_cells", C.c_int), ("n_u", C.c_int), ("n_p", C.c_int), ("n_T", C.c_int),
        ("temperature_degree", C.c_int),
        ("cell_nse_dofs", C.POINTER(C.c_int32)), ("cell_T_dofs", C.POINTER(C.c_int32)),
        ("cell_geometry", C.POINTER(C.c_double)), ("cell_diameter", C.POINTER(C.c_double)),
        ("nse", Constraints), ("T", Constraints),
    ]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p,
                           C.POINTER(C.c_size_t))


class HostComm(C.Structure):
    """dcp_host_comm: the caller's communicator for the distributed upload's
    host-side exchanges (the reference binds MPI_Allgather / MPI_Alltoallv)."""
    _fields_ = [("user", C.c_void_p), ("rank", C.c_int), ("world", C.c_int),
                ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


class Constraints64(C.Structure):
    _fields_ = [("n_lines", C.c_int64), ("line_dof", C.POINTER(C.c_int64)),
                ("entry_ptr", C.POINTER(C.c_int64)), ("entry_dof", C.POINTER(C.c_int64)),
                ("entry_w", C.POINTER(C.c_double)), ("inhomogeneity", C.POINTER(C.c_double))]


class DistMeshView(C.Structure):
    """dcp_dist_mesh: one rank's owned + ghost cells in global numbering."""
    _fields_ = [
        ("n_cells", C.c_int), ("n_owned_cells", C.c_int),
        ("cell_id", C.POINTER(C.c_int64)), ("cell_owner", C.POINTER(C.c_int32)),
        ("cell_nse_dofs", C.POINTER(C.c_int64)), ("cell_T_dofs", C.POINTER(C.c_int64)),
        ("cell_geometry", C.POINTER(C.c_double)), ("cell_diameter", C.POINTER(C.c_double)),
        ("n_u", C.c_int64), ("n_p", C.c_int64), ("n_T", C.c_int64),
        ("u_begin", C.c_int64), ("u_end", C.c_int64), ("p_begin", C.c_int64), ("p_end", C.c_int64),
        ("T_begin", C.c_int64), ("T_end", C.c_int64),
        ("nse", Constraints64), ("T", Constraints64),
    ]


class RunParams(C.Structure):
    _fields_ = [
        ("physics", Physics), ("initial_global_refinement", C.c_int),
        ("space_dimension", C.c_int), ("nse_velocity_degree", C.c_int),
        ("use_schur_complement_solver", C.c_int), ("use_FEEC_solver", C.c_int),
        ("adapt_time_step", C.c_int), ("final_time", C.c_double), ("R0", C.c_double),
        ("R1", C.c_double), ("length", C.c_double),
        ("use_block_preconditioner_feec", C.c_int), ("correct_pressure_to_zero_mean", C.c_int),
        ("solver_diagnostics_level", C.c_int), ("use_direct_solver", C.c_int),
    ]


class RunReport(C.Structure):
    """dcp_run_report: one time step of dcp_run (and the run totals)."""
    _fields_ = [
        ("timestep_number", C.c_int), ("steps", C.c_int), ("time_index", C.c_double),
        ("time_step", C.c_double), ("cfl", C.c_double), ("max_velocity", C.c_double),
        ("fgmres_outer", C.c_int), ("schur_inner", C.c_int), ("T_cg", C.c_int),
        ("total_outer", C.c_long), ("total_inner", C.c_long), ("total_T_cg", C.c_long),
        ("T_min", C.c_double), ("T_max", C.c_double),
    ]


STEP_CALLBACK = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(RunReport))


def load_library(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the hot path has no CPU fallback)")
    lib = C.CDLL(path)
    if not hasattr(lib, "dcp_abi_version") or lib.dcp_abi_version() != ABI_VERSION:
        raise ImportError(f"{path}: ABI version {getattr(lib, 'dcp_abi_version', lambda: '?')()}"
                          f" != {ABI_VERSION} (rebuild libdcp.so against include/dcp.h)")
    P, D, I = C.c_void_p, C.POINTER(C.c_double), C.c_int
    lib.dcp_last_error.restype = C.c_char_p
    lib.dcp_last_error.argtypes = [P]
    lib.dcp_ctx_create.argtypes = [C.POINTER(Config), C.POINTER(P)]
    lib.dcp_ctx_destroy.argtypes = [P]
    lib.dcp_ctx_destroy.restype = None
    lib.dcp_set_physics.argtypes = [P, C.POINTER(Physics)]
    lib.dcp_set_time_step.argtypes = [P, C.c_double]
    lib.dcp_set_option.argtypes = [P, I, I]
    lib.dcp_mesh_upload.argtypes = [P, I, P, P, P, P, I, I, I, C.POINTER(Constraints),
                                    C.POINTER(Constraints)]
    lib.dcp_mesh_check.argtypes = [I, P, P, P, P, I, I, I, C.POINTER(Constraints),
                                   C.POINTER(Constraints), C.POINTER(I)]
    lib.dcp_state_set.argtypes = [P, I, P, C.c_size_t]
    lib.dcp_state_get.argtypes = [P, I, P, C.c_size_t]
    lib.dcp_state_copy.argtypes = [P, I, I]
    lib.dcp_state_device_ptr.argtypes = [P, I]
    lib.dcp_state_device_ptr.restype = C.c_void_p
    for f in ("dcp_build_nse_preconditioner", "dcp_assemble_temperature_matrix",
              "dcp_assemble_temperature_rhs", "dcp_advance_state"):
        getattr(lib, f).argtypes = [P]
    lib.dcp_assemble_nse_system.argtypes = [P, I]
    lib.dcp_solve_nse.argtypes = [P, C.POINTER(I), C.POINTER(I)]
    lib.dcp_solve_nse_schur.argtypes = [P, C.POINTER(I), C.POINTER(I)]
    lib.dcp_solve_temperature.argtypes = [P, C.POINTER(I), D]
    lib.dcp_max_velocity.argtypes = [P, D]
    lib.dcp_cfl_number.argtypes = [P, D]
    lib.dcp_nse_vmult.argtypes = [P, P, P]
    lib.dcp_velocity_vmult.argtypes = [P, P, P]
    lib.dcp_mesh_geometry_info.argtypes = [C.c_int, P, P, P, P]
    lib.dcp_run.argtypes = [P, C.POINTER(RunParams), C.c_int, STEP_CALLBACK, P, C.POINTER(RunReport)]
    lib.dcp_schur_vmult.argtypes = [P, P, P]
    lib.dcp_block_preconditioner_vmult.argtypes = [P, P, P, I, C.POINTER(I)]
    lib.dcp_nse_matrix_export.argtypes = [P, C.POINTER(C.c_int64), P, P, P]
    lib.dcp_T_matrix_export.argtypes = [P, C.POINTER(C.c_int64), P, P, P]
    lib.dcp_precond_diagonals.argtypes = [P, P, P]
    lib.dcp_cell_nse_system.argtypes = [P, I, I, P, P]
    lib.dcp_get_timings.argtypes = [P, C.POINTER(Timings)]
    lib.dcp_pattern_info.argtypes = [P] + [C.POINTER(C.c_int64)] * 5
    lib.dcp_schur_layout.argtypes = [P, C.POINTER(C.c_int), C.POINTER(C.c_int64),
                                     C.POINTER(C.c_int)]
    lib.dcp_assembly_layout.argtypes = [P, P]
    lib.dcp_scatter_info.argtypes = [P, P, P, P]
    lib.dcp_matrix_powers_info.argtypes = [P, P]
    lib.dcp_device_memory.argtypes = [P, P]
    lib.dcp_comm_info.argtypes = [P, P]
    lib.dcp_local_sizes.argtypes = [P, P]
    lib.dcp_halo_selftest.argtypes = [P, I, P, I, P, P, I]
    lib.dcp_allreduce_selftest.argtypes = [P, P, C.c_size_t, I, C.POINTER(C.c_double)]
    lib.dcp_nse_coupling_export.argtypes = [P, I, C.POINTER(C.c_int64), P, P, P]
    lib.dcp_feec_partition_info.argtypes = [C.POINTER(FeecMeshView), I, I, I, P, P, P, P, P, P]
    lib.dcp_mesh2d_partition_info.argtypes = [C.POINTER(Mesh2DView), I, I, I, P, P, P, P, P, P]
    lib.dcp_time_operator.argtypes = [P, I, I, I, C.c_void_p, C.c_void_p, D]
    lib.dcp_host_mesh_create.argtypes = [I, I, C.c_double, C.c_double, C.c_double, I, I, I]
    lib.dcp_host_mesh_create.restype = P
    lib.dcp_host_mesh_renumber_cuthill_mckee.argtypes = [P]
    lib.dcp_host_mesh_renumber_dealii.argtypes = [P, P]
    lib.dcp_host_mesh_destroy.argtypes = [P]
    lib.dcp_host_mesh_destroy.restype = None
    lib.dcp_host_mesh_view_get.argtypes = [P, C.POINTER(MeshView)]
    lib.dcp_host_mesh_initial_temperature.argtypes = [P, P]
    lib.dcp_prm_load.argtypes = [C.c_char_p, C.POINTER(RunParams), C.c_char_p, I]
    lib.dcp_host_feec_view_get.argtypes = [P, C.POINTER(FeecMeshView)]
    lib.dcp_feec_mesh_upload.argtypes = [P, C.POINTER(FeecMeshView)]
    for f in ("dcp_feec_assemble_nse_system", "dcp_feec_build_nse_preconditioner"):
        getattr(lib, f).argtypes = [P]
    lib.dcp_feec_solve_nse.argtypes = [P, C.POINTER(I)]
    lib.dcp_feec_cell_system.argtypes = [P, I, I, P, P]
    lib.dcp_feec_matrix_export.argtypes = [P, I, C.POINTER(C.c_int64), P, P, P]
    lib.dcp_nccl_unique_id.argtypes = [P]
    lib.dcp_group_create.argtypes = [I]
    lib.dcp_group_create.restype = P
    lib.dcp_group_destroy.argtypes = [P]
    lib.dcp_group_destroy.restype = None
    lib.dcp_partition_info.argtypes = [I, P, P, P, P, I, I, I, C.POINTER(Constraints),
                                       C.POINTER(Constraints), I, I, P, P, P, P, P, P]
    lib.dcp_write_vtu.argtypes = [C.POINTER(MeshView), P, P, I, C.c_char_p]
    lib.dcp_write_pvtu_record.argtypes = [C.c_char_p, I, C.POINTER(C.c_char_p)]
    lib.dcp_write_feec_vtu.argtypes = [C.POINTER(FeecMeshView), P, P, I, C.c_char_p]
    lib.dcp_write_feec_pvtu_record.argtypes = [C.c_char_p, I, C.POINTER(C.c_char_p)]
    lib.dcp_solver_history.argtypes = [P, I, P, P, I, C.POINTER(I), C.POINTER(I)]
    lib.dcp_timer_summary.argtypes = [P, C.c_char_p, I]
    lib.dcp_timer_section.argtypes = [P, C.c_char_p, C.POINTER(C.c_long), C.POINTER(C.c_double)]
    lib.dcp_timer_record.argtypes = [P, C.c_char_p, C.c_double]
    lib.dcp_timer_reset.argtypes = [P]
    lib.dcp_mesh2d_upload.argtypes = [P, C.POINTER(Mesh2DView)]
    lib.dcp_mesh2d_check.argtypes = [C.POINTER(Mesh2DView), C.POINTER(I)]
    lib.dcp_host_mesh2d_create.argtypes = [I, C.c_double, C.c_double, C.c_double, I, I]
    lib.dcp_host_mesh2d_create.restype = P
    lib.dcp_host_mesh2d_view_get.argtypes = [P, C.POINTER(Mesh2DView), C.POINTER(D), C.POINTER(I)]
    lib.dcp_mesh_upload_distributed.argtypes = [P, C.POINTER(DistMeshView), C.POINTER(HostComm)]
    lib.dcp_dist_partition_info.argtypes = [C.POINTER(DistMeshView), C.POINTER(HostComm), P, P, P,
                                            P, P, P]
    lib.dcp_dist_partition_info_field.argtypes = [C.POINTER(DistMeshView), C.POINTER(HostComm), I,
                                                  P, P, P, P, P, P]
    lib.dcp_partition_info_field.argtypes = [I, P, P, P, P, I, I, I, C.POINTER(Constraints),
                                             C.POINTER(Constraints), I, I, I, P, P, P, P, P, P]
    lib.dcp_state_set_owned.argtypes = [P, I, P, C.c_size_t]
    lib.dcp_state_get_owned.argtypes = [P, I, P, C.c_size_t]
    return lib


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = load_library()
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _arr(p, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dtype, copy=True)


class ConstraintSet:
    """A closed AffineConstraints object (numpy arrays)."""

    def __init__(self, line_dof, entry_ptr, entry_dof, entry_w, inhomogeneity):
        self.line_dof = np.ascontiguousarray(line_dof, dtype=np.int32)
        self.entry_ptr = np.ascontiguousarray(entry_ptr, dtype=np.int32)
        self.entry_dof = np.ascontiguousarray(entry_dof, dtype=np.int32)
        self.entry_w = np.ascontiguousarray(entry_w, dtype=np.float64)
        self.inhomogeneity = np.ascontiguousarray(inhomogeneity, dtype=np.float64)

    @classmethod
    def from_view(cls, v: Constraints):
        n = v.n_lines
        ptr = _arr(v.entry_ptr, n + 1, np.int32)
        ne = int(ptr[-1]) if n else 0
        if n == 0:
            ptr = np.zeros(1, np.int32)
        return cls(_arr(v.line_dof, n, np.int32), ptr, _arr(v.entry_dof, ne, np.int32),
                   _arr(v.entry_w, ne, np.float64), _arr(v.inhomogeneity, n, np.float64))

    def as_struct(self) -> Constraints:
        s = Constraints()
        s.n_lines = len(self.line_dof)
        s.line_dof = self.line_dof.ctypes.data_as(C.POINTER(C.c_int))
        s.entry_ptr = self.entry_ptr.ctypes.data_as(C.POINTER(C.c_int))
        s.entry_dof = self.entry_dof.ctypes.data_as(C.POINTER(C.c_int))
        s.entry_w = self.entry_w.ctypes.data_as(C.POINTER(C.c_double))
        s.inhomogeneity = self.inhomogeneity.ctypes.data_as(C.POINTER(C.c_double))
        return s


class HostMesh:
    """Refined shell / cube with DoFs and constraints (setup_dofs restated)."""

    NORMAL_MODES = ("mapping", "radial", "consistent")  # dcp_host_mesh_create normal_mode

    def __init__(self, cuboid=False, refine=2, R0=1.0, R1=3.0, length=1.0, temperature_degree=1,
                 normals="mapping", feec=False, mapping_q_on_all_cells=False,
                 cuthill_mckee=False, dealii_order=False):
        """cuthill_mckee: renumber the NSE dofs as setup_dofs does for the
        Schur-complement solver (dcp_host_mesh_renumber_cuthill_mckee).
        dealii_order: number the NSE and temperature dofs in deal.II's
        distribute_dofs order on the 6-cell hyper_shell first
        (dcp_host_mesh_renumber_dealii); `dealii_cells` then holds the mesh cell
        of each deal.II active cell."""
        if normals not in self.NORMAL_MODES:
            raise ValueError("normals must be one of %s" % (self.NORMAL_MODES,))
        h = lib().dcp_host_mesh_create(int(cuboid), int(refine), float(R0), float(R1),
                                       float(length), int(temperature_degree),
                                       self.NORMAL_MODES.index(normals),
                                       int(bool(mapping_q_on_all_cells)))
        if not h:
            raise DcpError(DCP_ERR_INVALID, lib().dcp_last_error(None).decode())
        try:
            self.dealii_cells = None
            if dealii_order:
                cells = np.zeros(6 * 8 ** int(refine), dtype=np.int32)
                if lib().dcp_host_mesh_renumber_dealii(h, _ptr(cells)) != DCP_OK:
                    raise DcpError(DCP_ERR_INVALID, lib().dcp_last_error(None).decode())
                self.dealii_cells = cells
            if cuthill_mckee and lib().dcp_host_mesh_renumber_cuthill_mckee(h) != DCP_OK:
                raise DcpError(DCP_ERR_INVALID, lib().dcp_last_error(None).decode())
            v = MeshView()
            lib().dcp_host_mesh_view_get(h, C.byref(v))
            self.n_cells, self.n_u, self.n_p, self.n_T = v.n_cells, v.n_u, v.n_p, v.n_T
            self.n_vnodes = v.n_vnodes
            self.cell_nse_dofs = _arr(v.cell_nse_dofs, self.n_cells * 89, np.int32).reshape(-1, 89)
            tdpc = 8 if temperature_degree == 1 else 27
            self.cell_T_dofs = _arr(v.cell_T_dofs, self.n_cells * tdpc, np.int32).reshape(-1, tdpc)
            # MappingQ(3) support points per cell (64, lexicographic, Gauss-Lobatto)
            self.cell_geometry = _arr(v.cell_geometry, self.n_cells * 192,
                                      np.float64).reshape(-1, 64, 3)
            self.cell_diameter = _arr(v.cell_diameter, self.n_cells, np.float64)
            self.node_xyz = _arr(v.node_xyz, self.n_vnodes * 3, np.float64).reshape(-1, 3)
            self.nse_constraints = ConstraintSet.from_view(v.nse)
            self.T_constraints = ConstraintSet.from_view(v.T)
            self.T0 = np.zeros(self.n_T)
            lib().dcp_host_mesh_initial_temperature(h, _ptr(self.T0))
            self.feec = FeecTopology(h, self) if feec else None
        finally:
            lib().dcp_host_mesh_destroy(h)
        self.cuboid = bool(cuboid)
        self.refine = refine
        self.temperature_degree = temperature_degree
        self.mapping_q_on_all_cells = bool(mapping_q_on_all_cells)

    def write_vtu(self, path, nse_solution, T_solution, partition=0):
        """output_results' DataOut::write_vtu of the joint [u p T] solution
        (dcp_write_vtu; host-only, classic Q2/Q1 mesh)."""
        v = MeshView()
        v.n_cells, v.n_u, v.n_p, v.n_T = self.n_cells, self.n_u, self.n_p, self.n_T
        v.cell_nse_dofs = self.cell_nse_dofs.ctypes.data_as(C.POINTER(C.c_int32))
        v.cell_T_dofs = self.cell_T_dofs.ctypes.data_as(C.POINTER(C.c_int32))
        v.cell_geometry = self.cell_geometry.ctypes.data_as(C.POINTER(C.c_double))
        u = np.ascontiguousarray(nse_solution, dtype=np.float64)
        T = np.ascontiguousarray(T_solution, dtype=np.float64)
        if u.size != self.n_u + self.n_p or T.size != self.n_T:
            raise ValueError("solution sizes do not match the mesh")
        rc = lib().dcp_write_vtu(C.byref(v), _ptr(u), _ptr(T), int(partition), str(path).encode())
        if rc != DCP_OK:
            raise DcpError(rc, "dcp_write_vtu failed for " + str(path))

    def check(self, nse_constraints=None, T_constraints=None):
        """Host-only validation of the device upload; returns the number of
        cell colours or raises DcpError (e.g. periodic constraints)."""
        nc = (nse_constraints or self.nse_constraints).as_struct()
        tc = (T_constraints or self.T_constraints).as_struct()
        ncol = C.c_int(0)
        rc = lib().dcp_mesh_check(self.n_cells, _ptr(self.cell_nse_dofs), _ptr(self.cell_T_dofs),
                                  _ptr(self.cell_geometry), _ptr(self.cell_diameter), self.n_u,
                                  self.n_p, self.n_T, C.byref(nc), C.byref(tc), C.byref(ncol))
        if rc != DCP_OK:
            raise DcpError(rc, lib().dcp_last_error(None).decode())
        return ncol.value

    def geometry_info(self):
        """Host-only: (separable, n_columns, n_layers) of the radially separable
        MappingQ(3) geometry the matrix-free operator uses (dcp_mesh_geometry_info)."""
        sep, nc, nl = C.c_int(0), C.c_int(0), C.c_int(0)
        rc = lib().dcp_mesh_geometry_info(self.n_cells, _ptr(self.cell_geometry), C.byref(sep),
                                          C.byref(nc), C.byref(nl))
        if rc != DCP_OK:
            raise DcpError(rc, lib().dcp_last_error(None).decode())
        return bool(sep.value), nc.value, nl.value


class HostMesh2D:
    """The 2D shell of Standard::BoussinesqModel<2> (dcp_host_mesh2d_create):
    hyper_shell<2> with 12 cells, refine_global, FESystem(FE_Q(2)^2, FE_Q(1))
    DoFs (22 per cell), FE_Q(temperature_degree) temperature, constraints."""

    dim = 2

    def __init__(self, refine=2, R0=1.0, R1=3.0, length=1.0, temperature_degree=2,
                 mapping_q_on_all_cells=False, cuthill_mckee=False):
        h = lib().dcp_host_mesh2d_create(int(refine), float(R0), float(R1), float(length),
                                         int(temperature_degree), int(bool(mapping_q_on_all_cells)))
        if not h:
            raise DcpError(DCP_ERR_INVALID, lib().dcp_last_error(None).decode())
        try:
            if cuthill_mckee and lib().dcp_host_mesh_renumber_cuthill_mckee(h) != DCP_OK:
                raise DcpError(DCP_ERR_INVALID, lib().dcp_last_error(None).decode())
            v = Mesh2DView()
            xy = C.POINTER(C.c_double)()
            nv = C.c_int(0)
            rc = lib().dcp_host_mesh2d_view_get(h, C.byref(v), C.byref(xy), C.byref(nv))
            if rc != DCP_OK:
                raise DcpError(rc, "dcp_host_mesh2d_view_get failed")
            nc = v.n_cells
            self.n_cells, self.n_u, self.n_p, self.n_T = nc, v.n_u, v.n_p, v.n_T
            self.n_vnodes = nv.value
            self.temperature_degree = v.temperature_degree
            tdpc = (self.temperature_degree + 1) ** 2
            self.cell_nse_dofs = _arr(v.cell_nse_dofs, nc * 22, np.int32).reshape(-1, 22)
            self.cell_T_dofs = _arr(v.cell_T_dofs, nc * tdpc, np.int32).reshape(-1, tdpc)
            # MappingQ(3) support points per cell (16, lexicographic, Gauss-Lobatto)
            self.cell_geometry = _arr(v.cell_geometry, nc * 32, np.float64).reshape(-1, 16, 2)
            self.cell_diameter = _arr(v.cell_diameter, nc, np.float64)
            self.node_xy = _arr(xy, self.n_vnodes * 2, np.float64).reshape(-1, 2)
            self.nse_constraints = ConstraintSet.from_view(v.nse)
            self.T_constraints = ConstraintSet.from_view(v.T)
            self.T0 = np.zeros(self.n_T)
            lib().dcp_host_mesh_initial_temperature(h, _ptr(self.T0))
        finally:
            lib().dcp_host_mesh_destroy(h)
        self.refine = refine
        self.mapping_q_on_all_cells = bool(mapping_q_on_all_cells)

    def as_struct(self, nse_constraints=None, T_constraints=None):
        v = Mesh2DView()
        v.n_cells, v.n_u, v.n_p, v.n_T = self.n_cells, self.n_u, self.n_p, self.n_T
        v.temperature_degree = self.temperature_degree
        v.cell_nse_dofs = self.cell_nse_dofs.ctypes.data_as(C.POINTER(C.c_int32))
        v.cell_T_dofs = self.cell_T_dofs.ctypes.data_as(C.POINTER(C.c_int32))
        v.cell_geometry = self.cell_geometry.ctypes.data_as(C.POINTER(C.c_double))
        v.cell_diameter = self.cell_diameter.ctypes.data_as(C.POINTER(C.c_double))
        self._nc = (nse_constraints or self.nse_constraints).as_struct()
        self._tc = (T_constraints or self.T_constraints).as_struct()
        v.nse, v.T = self._nc, self._tc
        return v

    def check(self, nse_constraints=None, T_constraints=None):
        """Host-only validation of the 2D upload; returns the number of cell colours."""
        v = self.as_struct(nse_constraints, T_constraints)
        ncol = C.c_int(0)
        rc = lib().dcp_mesh2d_check(C.byref(v), C.byref(ncol))
        if rc != DCP_OK:
            raise DcpError(rc, lib().dcp_last_error(None).decode())
        return ncol.value


class FeecTopology:
    """FEEC DoFs of a host mesh (dcp_host_feec_view_get): Nedelec edges (w),
    Raviart-Thomas faces (u), DGQ0 cells (p), with orientation signs."""

    def __init__(self, h, mesh):
        v = FeecMeshView()
        rc = lib().dcp_host_feec_view_get(h, C.byref(v))
        if rc != DCP_OK:
            raise DcpError(rc, lib().dcp_last_error(None).decode())
        nc = v.n_cells
        self.n_cells, self.n_w, self.n_u, self.n_p, self.n_T = nc, v.n_w, v.n_u, v.n_p, v.n_T
        self.cell_w = _arr(v.cell_w, nc * 12, np.int32).reshape(-1, 12)
        self.sign_w = _arr(v.sign_w, nc * 12, np.int8).reshape(-1, 12)
        self.cell_u = _arr(v.cell_u, nc * 6, np.int32).reshape(-1, 6)
        self.sign_u = _arr(v.sign_u, nc * 6, np.int8).reshape(-1, 6)
        self.cell_vertices = _arr(v.cell_vertices, nc * 24, np.float64).reshape(-1, 8, 3)
        self.cell_diameter = _arr(v.cell_diameter, nc, np.float64)
        self.cell_T_dofs = _arr(v.cell_T_dofs, nc * 8, np.int32).reshape(-1, 8)
        self.w_fixed = _arr(v.w_fixed, self.n_w, np.uint8)
        self.u_fixed = _arr(v.u_fixed, self.n_u, np.uint8)
        self.T_constraints = mesh.T_constraints
        self.n = self.n_w + self.n_u + self.n_p
        # global [w | u | p] dofs of each cell's 19 local dofs and their signs
        self.cell_dofs = np.concatenate(
            [self.cell_w, self.n_w + self.cell_u,
             (self.n_w + self.n_u + np.arange(nc, dtype=np.int32))[:, None]], axis=1)
        self.signs = np.concatenate([self.sign_w, self.sign_u, np.ones((nc, 1), np.int8)], axis=1)
        self.fixed = np.concatenate([self.w_fixed, self.u_fixed, np.zeros(self.n_p, np.uint8)])

    def write_vtu(self, path, nse_solution, T_solution, partition=0):
        """The FEEC model's output_results (dcp_write_feec_vtu; host-only):
        one hexahedron per cell, vorticity / velocity / p / T / partition at
        its vertices."""
        x = np.ascontiguousarray(nse_solution, dtype=np.float64)
        T = np.ascontiguousarray(T_solution, dtype=np.float64)
        if x.size != self.n or T.size != self.n_T:
            raise ValueError("solution sizes do not match the FEEC mesh")
        v = self.as_struct()
        rc = lib().dcp_write_feec_vtu(C.byref(v), _ptr(x), _ptr(T), int(partition),
                                      str(path).encode())
        if rc != DCP_OK:
            raise DcpError(rc, "dcp_write_feec_vtu failed for " + str(path))

    def as_struct(self):
        v = FeecMeshView()
        v.n_cells, v.n_w, v.n_u, v.n_p, v.n_T = self.n_cells, self.n_w, self.n_u, self.n_p, self.n_T
        for name, arr, ct in (("cell_w", self.cell_w, C.c_int32), ("sign_w", self.sign_w, C.c_int8),
                              ("cell_u", self.cell_u, C.c_int32), ("sign_u", self.sign_u, C.c_int8),
                              ("cell_vertices", self.cell_vertices, C.c_double),
                              ("cell_diameter", self.cell_diameter, C.c_double),
                              ("cell_T_dofs", self.cell_T_dofs, C.c_int32),
                              ("w_fixed", self.w_fixed, C.c_uint8),
                              ("u_fixed", self.u_fixed, C.c_uint8)):
            setattr(v, name, arr.ctypes.data_as(C.POINTER(ct)))
        self._tc = self.T_constraints.as_struct()
        v.T = self._tc
        return v


def torch_host_comm(group=None):
    """A dcp_host_comm over an initialised torch.distributed process group
    (gloo on the host; any backend whose collectives take CPU tensors)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)

    def allgather(_user, send, nbytes, recv):
        try:
            src = np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(nbytes,)) \
                if nbytes else np.zeros(0, np.uint8)
            t = torch.from_numpy(src.copy())
            out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(out, t, group=group)
            if nbytes:
                flat = torch.cat(out).numpy()   # kept alive across the copy
                C.memmove(recv, flat.ctypes.data, nbytes * world)
            return 0
        except Exception:  # noqa: BLE001 - reported to the library as a failure
            return 1

    def alltoallv(_user, send, send_bytes, recv, recv_bytes):
        try:
            sb = [int(send_bytes[k]) for k in range(world)]
            rb = [int(recv_bytes[k]) for k in range(world)]
            src = np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(sum(sb),)) \
                if sum(sb) else np.zeros(0, np.uint8)
            out = torch.empty(sum(rb), dtype=torch.uint8)
            dist.all_to_all_single(out, torch.from_numpy(src.copy()), output_split_sizes=rb,
                                   input_split_sizes=sb, group=group)
            if sum(rb):
                flat = out.numpy()
                C.memmove(recv, flat.ctypes.data, sum(rb))
            return 0
        except Exception:  # noqa: BLE001
            return 1

    hc = HostComm(None, rank, world, ALLGATHER_FN(allgather), ALLTOALLV_FN(alltoallv))
    hc._keep = (hc.allgather, hc.alltoallv)
    return hc


class ThreadHostComms:
    """dcp_host_comm for `world` ranks of ONE process, one thread per rank (the
    in-process groups of the tests): the collectives meet on a barrier and
    exchange bytes through shared slots. comm(rank) is that rank's HostComm."""

    def __init__(self, world):
        import threading
        self.world = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world
        self._comms = {}

    def comm(self, rank):
        if rank in self._comms:
            return self._comms[rank]
        world = self.world

        def allgather(_user, send, nbytes, recv):
            try:
                self.slots[rank] = C.string_at(send, nbytes) if nbytes else b""
                self.bar.wait()
                if nbytes:
                    C.memmove(recv, b"".join(self.slots), nbytes * world)
                self.bar.wait()
                return 0
            except Exception:  # noqa: BLE001 - reported to the library as a failure
                return 1

        def alltoallv(_user, send, send_bytes, recv, recv_bytes):
            try:
                sb = [int(send_bytes[k]) for k in range(world)]
                data = C.string_at(send, sum(sb)) if sum(sb) else b""
                off = np.concatenate([[0], np.cumsum(sb)]).astype(int)
                self.slots[rank] = [data[off[k]:off[k + 1]] for k in range(world)]
                self.bar.wait()
                out = b"".join(self.slots[k][rank] for k in range(world))
                if out:
                    C.memmove(recv, out, len(out))
                self.bar.wait()
                return 0
            except Exception:  # noqa: BLE001
                return 1

        hc = HostComm(None, rank, world, ALLGATHER_FN(allgather), ALLTOALLV_FN(alltoallv))
        hc._keep = (hc.allgather, hc.alltoallv)
        self._comms[rank] = hc
        return hc


class DistMesh:
    """One rank's part of a distributed mesh (dcp_dist_mesh), built here from a
    global HostMesh the way a p4est run would hold it: the rank's owned cells
    (an equal split in tree order), its ghost cells (one vertex layer), DoFs
    renumbered so every rank owns one contiguous range per block (what deal.II's
    distribute_dofs + component_wise give), owner = rank of the lowest-index
    cell touching the DoF. `perm_*` map the HostMesh numbering to this one."""

    def __init__(self, m: HostMesh, rank: int, world: int):
        nc, nv = m.n_cells, m.n_u // 3
        start = [r * nc // world for r in range(world + 1)]
        cell_rank = np.zeros(nc, np.int32)
        for r in range(world):
            cell_rank[start[r]:start[r + 1]] = r
        vel = m.cell_nse_dofs[:, [4 * t for t in range(8)] + [32 + 3 * t for t in range(19)]] // 3
        pre = m.cell_nse_dofs[:, [4 * t + 3 for t in range(8)]] - m.n_u
        tdo = m.cell_T_dofs

        def owners(ents, n):
            own = np.full(n, world, np.int32)
            for c in range(nc):   # lowest-index cell touching the entity
                e = ents[c]
                own[e] = np.minimum(own[e], cell_rank[c])
            return own

        vown, pown, Town = owners(vel, nv), owners(pre, m.n_p), owners(tdo, m.n_T)

        def renumber(own):
            order = np.lexsort((np.arange(len(own)), own))    # by (owner, old id)
            new = np.empty(len(own), np.int64)
            new[order] = np.arange(len(own))
            bounds = np.searchsorted(own[order], np.arange(world + 1))
            return new, bounds

        self.perm_v, vb = renumber(vown)
        self.perm_p, pb = renumber(pown)
        self.perm_T, tb = renumber(Town)
        n_u = m.n_u
        perm_nse = np.empty(n_u + m.n_p, np.int64)
        perm_nse[:n_u] = 3 * np.repeat(self.perm_v, 3) + np.tile(np.arange(3), nv)
        perm_nse[n_u:] = n_u + self.perm_p
        self.perm_nse = perm_nse
        # owned cells + one vertex layer of ghosts
        vcells = [[] for _ in range(m.n_p)]
        for c in range(nc):
            for p in pre[c]:
                vcells[p].append(c)
        owned = list(range(start[rank], start[rank + 1]))
        ghost = sorted({o for c in owned for p in pre[c] for o in vcells[p]} - set(owned))
        cells = np.array(owned + ghost, np.int64)
        self.cells = cells
        self.rank, self.world = rank, world
        self.n_cells, self.n_owned_cells = len(cells), len(owned)
        self.cell_id = cells.copy()
        self.cell_owner = cell_rank[cells].astype(np.int32)
        self.cell_nse_dofs = perm_nse[m.cell_nse_dofs[cells]].astype(np.int64)
        self.cell_T_dofs = self.perm_T[m.cell_T_dofs[cells]].astype(np.int64)
        self.cell_geometry = np.ascontiguousarray(m.cell_geometry[cells])
        self.cell_diameter = np.ascontiguousarray(m.cell_diameter[cells])
        self.n_u, self.n_p, self.n_T = m.n_u, m.n_p, m.n_T
        self.u_begin, self.u_end = 3 * int(vb[rank]), 3 * int(vb[rank + 1])
        self.p_begin, self.p_end = n_u + int(pb[rank]), n_u + int(pb[rank + 1])
        self.T_begin, self.T_end = int(tb[rank]), int(tb[rank + 1])
        # constraint lines of the locally relevant dofs, global (renumbered) ids
        rel_nse = np.unique(self.cell_nse_dofs)
        rel_T = np.unique(self.cell_T_dofs)
        self.nse_lines = self._lines(m.nse_constraints, perm_nse, rel_nse)
        self.T_lines = self._lines(m.T_constraints, self.perm_T, rel_T)

    @staticmethod
    def _lines(cs, perm, relevant):
        keep = np.isin(perm[cs.line_dof], relevant)
        line, ptr, edof, w, inh = [], [0], [], [], []
        for l in np.nonzero(keep)[0]:
            line.append(perm[cs.line_dof[l]])
            inh.append(cs.inhomogeneity[l])
            for k in range(cs.entry_ptr[l], cs.entry_ptr[l + 1]):
                edof.append(perm[cs.entry_dof[k]])
                w.append(cs.entry_w[k])
            ptr.append(len(edof))
        return (np.array(line, np.int64), np.array(ptr, np.int64), np.array(edof, np.int64),
                np.array(w, np.float64), np.array(inh, np.float64))

    def as_struct(self) -> DistMeshView:
        v = DistMeshView()
        v.n_cells, v.n_owned_cells = self.n_cells, self.n_owned_cells
        for name, ct in (("cell_id", C.c_int64), ("cell_owner", C.c_int32),
                         ("cell_nse_dofs", C.c_int64), ("cell_T_dofs", C.c_int64),
                         ("cell_geometry", C.c_double), ("cell_diameter", C.c_double)):
            setattr(v, name, getattr(self, name).ctypes.data_as(C.POINTER(ct)))
        v.n_u, v.n_p, v.n_T = self.n_u, self.n_p, self.n_T
        v.u_begin, v.u_end, v.p_begin, v.p_end = self.u_begin, self.u_end, self.p_begin, self.p_end
        v.T_begin, v.T_end = self.T_begin, self.T_end
        for field, lines in (("nse", self.nse_lines), ("T", self.T_lines)):
            c = Constraints64()
            c.n_lines = len(lines[0])
            for name, arr, ct in zip(("line_dof", "entry_ptr", "entry_dof", "entry_w", "inhomogeneity"),
                                     lines, (C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_double)):
                setattr(c, name, arr.ctypes.data_as(C.POINTER(ct)))
            setattr(v, field, c)
        return v

    def owned_nse(self, global_vec):
        """This rank's owned entries of an NSE vector in the HostMesh numbering,
        in the distributed numbering's ascending order."""
        g = np.empty_like(global_vec)
        g[self.perm_nse] = global_vec
        return np.concatenate([g[self.u_begin:self.u_end], g[self.p_begin:self.p_end]])

    def owned_T(self, global_vec):
        g = np.empty_like(global_vec)
        g[self.perm_T] = global_vec
        return g[self.T_begin:self.T_end].copy()


def dist_partition_info(dm: DistMesh, comm: HostComm, field: str = "v"):
    """dcp_dist_partition_info_field on this rank (host only; every rank calls
    it): sizes and the halo lists (global ids) of `field` ("v" velocity
    support points, "p" pressure, "T" temperature) per peer."""
    fid = {"v": 0, "p": 1, "T": 2}[field]
    view = dm.as_struct()
    info = np.zeros(12, np.int64)
    rc = lib().dcp_dist_partition_info_field(C.byref(view), C.byref(comm), fid, _ptr(info), None,
                                             None, None, None, None)
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    npeer, ns, nr = int(info[8]), int(info[9]), int(info[10])
    peers = np.zeros(max(npeer, 1), np.int32)
    sp, rp = np.zeros(npeer + 1, np.int32), np.zeros(npeer + 1, np.int32)
    sg, rg = np.zeros(max(ns, 1), np.int64), np.zeros(max(nr, 1), np.int64)
    rc = lib().dcp_dist_partition_info_field(C.byref(view), C.byref(comm), fid, _ptr(info), _ptr(peers),
                                       _ptr(sp), _ptr(sg), _ptr(rp), _ptr(rg))
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    keys = ("n_cells", "n_owned_cells", "nvo", "nvg", "npo", "npg", "nTo", "nTg", "n_peers",
            "n_send", "n_recv", "n_colors")
    out = {k: int(v) for k, v in zip(keys, info)}
    out["send"] = {int(p): sg[sp[i]:sp[i + 1]].copy() for i, p in enumerate(peers[:npeer])}
    out["recv"] = {int(p): rg[rp[i]:rp[i + 1]].copy() for i, p in enumerate(peers[:npeer])}
    return out


def load_prm(path: str) -> RunParams:
    rp = RunParams()
    err = C.create_string_buffer(512)
    rc = lib().dcp_prm_load(path.encode(), C.byref(rp), err, 512)
    if rc != DCP_OK:
        raise DcpError(rc, err.value.decode())
    return rp


def nccl_unique_id() -> bytes:
    """ncclUniqueId (128 bytes) for dcp_config.nccl_id; call on rank 0 only."""
    buf = C.create_string_buffer(128)
    rc = lib().dcp_nccl_unique_id(buf)
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    return buf.raw


class Group:
    """In-process group of world_size contexts on one device (dcp_group):
    drive each rank's Context from its own thread (tests of the multi-rank
    path on one GPU)."""

    def __init__(self, world_size):
        self.world_size = world_size
        self._h = lib().dcp_group_create(world_size)
        if not self._h:
            raise DcpError(DCP_ERR_DEVICE, lib().dcp_last_error(None).decode())

    def close(self):
        if self._h:
            lib().dcp_group_destroy(self._h)
            self._h = None


def partition_info(m, rank, world, field="v"):
    """Host-only summary of rank's partition (dcp_partition_info_field): a dict
    of sizes and the halo lists (global ids) of `field` ("v" velocity support
    points, "p" pressure, "T" temperature) per peer."""
    info = np.zeros(12, np.int64)
    nc, tc = m.nse_constraints.as_struct(), m.T_constraints.as_struct()
    args = (m.n_cells, _ptr(m.cell_nse_dofs), _ptr(m.cell_T_dofs), _ptr(m.cell_geometry),
            _ptr(m.cell_diameter), m.n_u, m.n_p, m.n_T, C.byref(nc), C.byref(tc), rank, world,
            {"v": 0, "p": 1, "T": 2}[field])
    rc = lib().dcp_partition_info_field(*args, _ptr(info), None, None, None, None, None)
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    npeer, ns, nr = int(info[8]), int(info[9]), int(info[10])
    peers = np.zeros(npeer, np.int32)
    sp, rp = np.zeros(npeer + 1, np.int32), np.zeros(npeer + 1, np.int32)
    sg, rg = np.zeros(max(ns, 1), np.int64), np.zeros(max(nr, 1), np.int64)
    rc = lib().dcp_partition_info_field(*args, _ptr(info), _ptr(peers), _ptr(sp), _ptr(sg),
                                        _ptr(rp), _ptr(rg))
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    keys = ("n_cells", "n_owned_cells", "nvo", "nvg", "npo", "npg", "nTo", "nTg", "n_peers",
            "n_send", "n_recv", "n_colors")
    out = {k: int(v) for k, v in zip(keys, info)}
    out["send"] = {int(p): sg[sp[i]:sp[i + 1]].copy() for i, p in enumerate(peers)}
    out["recv"] = {int(p): rg[rp[i]:rp[i + 1]].copy() for i, p in enumerate(peers)}
    return out


def feec_partition_info(m, rank, world, field):
    """Host-only summary of rank's FEEC partition (dcp_feec_partition_info) and
    the halo lists (global ids) per peer of `field` ("w", "u", "p", "T")."""
    fid = {"w": 0, "u": 1, "p": 2, "T": 3}[field]
    view = m.feec.as_struct()
    info = np.zeros(11, np.int64)
    rc = lib().dcp_feec_partition_info(C.byref(view), rank, world, fid, _ptr(info), None, None,
                                       None, None, None)
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    npeer, ns, nr = int(info[8]), int(info[9]), int(info[10])
    peers = np.zeros(max(npeer, 1), np.int32)
    sp, rp = np.zeros(npeer + 1, np.int32), np.zeros(npeer + 1, np.int32)
    sg, rg = np.zeros(max(ns, 1), np.int64), np.zeros(max(nr, 1), np.int64)
    rc = lib().dcp_feec_partition_info(C.byref(view), rank, world, fid, _ptr(info), _ptr(peers),
                                       _ptr(sp), _ptr(sg), _ptr(rp), _ptr(rg))
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    keys = ("n_cells", "n_owned_cells", "nwo", "nwg", "nuo", "nug", "nTo", "nTg", "n_peers",
            "n_send", "n_recv")
    out = {k: int(v) for k, v in zip(keys, info)}
    out["send"] = {int(p): sg[sp[i]:sp[i + 1]].copy() for i, p in enumerate(peers[:npeer])}
    out["recv"] = {int(p): rg[rp[i]:rp[i + 1]].copy() for i, p in enumerate(peers[:npeer])}
    return out


def mesh2d_partition_info(m, rank, world, field):
    """Host-only summary of rank's 2D partition (dcp_mesh2d_partition_info) and
    the halo lists (global ids) per peer of `field` ("u", "p", "T")."""
    fid = {"u": 0, "p": 1, "T": 2}[field]
    view = m.as_struct()
    info = np.zeros(11, np.int64)
    rc = lib().dcp_mesh2d_partition_info(C.byref(view), rank, world, fid, _ptr(info), None, None,
                                         None, None, None)
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    npeer, ns, nr = int(info[8]), int(info[9]), int(info[10])
    peers = np.zeros(max(npeer, 1), np.int32)
    sp, rp = np.zeros(npeer + 1, np.int32), np.zeros(npeer + 1, np.int32)
    sg, rg = np.zeros(max(ns, 1), np.int64), np.zeros(max(nr, 1), np.int64)
    rc = lib().dcp_mesh2d_partition_info(C.byref(view), rank, world, fid, _ptr(info), _ptr(peers),
                                         _ptr(sp), _ptr(sg), _ptr(rp), _ptr(rg))
    if rc != DCP_OK:
        raise DcpError(rc, lib().dcp_last_error(None).decode())
    keys = ("n_cells", "n_owned_cells", "nuo", "nug", "npo", "npg", "nTo", "nTg", "n_peers",
            "n_send", "n_recv")
    out = {k: int(v) for k, v in zip(keys, info)}
    out["send"] = {int(p): sg[sp[i]:sp[i + 1]].copy() for i, p in enumerate(peers[:npeer])}
    out["recv"] = {int(p): rg[rp[i]:rp[i + 1]].copy() for i, p in enumerate(peers[:npeer])}
    return out


class Context:
    """One GPU context (dcp_ctx). world_size > 1: pass nccl_id (the bytes of
    nccl_unique_id() from rank 0; one process per GPU) or group (Group)."""

    def __init__(self, device=0, rank=0, world_size=1, nccl_id=None, group=None):
        self._id = C.create_string_buffer(nccl_id, 128) if nccl_id is not None else None
        cfg = Config(device, rank, world_size,
                     C.cast(self._id, C.c_void_p) if self._id is not None else None,
                     group._h if group is not None else None)
        h = C.c_void_p()
        rc = lib().dcp_ctx_create(C.byref(cfg), C.byref(h))
        if rc != DCP_OK:
            raise DcpError(rc, lib().dcp_last_error(None).decode())
        self._h = h
        self.mesh = None

    def close(self):
        if self._h:
            lib().dcp_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, allow_not_converged=False):
        if rc == DCP_OK or (allow_not_converged and rc == DCP_NOT_CONVERGED):
            return rc
        raise DcpError(rc, lib().dcp_last_error(self._h).decode())

    # -- setup
    def set_physics(self, ph: Physics):
        self.physics = ph
        self._check(lib().dcp_set_physics(self._h, C.byref(ph)))

    def set_time_step(self, dt: float):
        self._check(lib().dcp_set_time_step(self._h, float(dt)))

    def set_schur_explicit(self, on: bool):
        """True: apply S = B D^-1 B^T as one formed CSR matrix (default);
        False: B^T, Jacobi, B as SchurComplement::vmult does."""
        self._check(lib().dcp_set_option(self._h, OPT_SCHUR_EXPLICIT, int(bool(on))))

    def set_matrix_free(self, mode):
        """True / 1 (default): solver products with nse_matrix / its A block are
        evaluated matrix-free (cell-order kernel + dof gather); 2: matrix-free
        in colour-class launches; False / 0: block-CSR SpMV of the assembled
        matrix."""
        self._check(lib().dcp_set_option(self._h, OPT_MATRIX_FREE, int(mode)))

    def set_inner_max_steps(self, n: int):
        """DCP_OPT_INNER_MAX_STEPS (probe hook): cap of the inner Schur GMRES
        (the reference's SolverControl(5000, ...))."""
        self._check(lib().dcp_set_option(self._h, OPT_INNER_MAX_STEPS, int(n)))

    def set_schur_fixed_inner(self, k: int):
        """DCP_OPT_SCHUR_FIXED_INNER (parity hook): the Schur-complement solver's
        inner CGs run exactly k steps (0 = the reference's 1e-6 rule)."""
        self._check(lib().dcp_set_option(self._h, OPT_SCHUR_FIXED_INNER, int(k)))

    def set_log_history(self, on: bool):
        """DCP_OPT_LOG_HISTORY: record the SolverControl checks of the NSE
        solve's FGMRES attempts (log_history = true, :1166-1169)."""
        self._check(lib().dcp_set_option(self._h, OPT_LOG_HISTORY, int(bool(on))))

    def solver_history(self, attempt=0):
        """(steps, residuals, result) of the last solve_nse's FGMRES attempt
        (0: FGMRES(30), 1: the do_solve_A FGMRES(50) fallback); result 0 =
        not run, 1 = convergence, 2 = failure."""
        n, res = C.c_int(0), C.c_int(0)
        self._check(lib().dcp_solver_history(self._h, int(attempt), None, None, 0, C.byref(n),
                                             C.byref(res)))
        steps, vals = np.zeros(n.value, np.int32), np.zeros(n.value)
        self._check(lib().dcp_solver_history(self._h, int(attempt), _ptr(steps), _ptr(vals),
                                             n.value, C.byref(n), C.byref(res)))
        return steps, vals, res.value

    def deallog(self, depth=2):
        """The solver lines deallog prints at depth_console(depth) >= 2:
        SolverFGMRES's prefix with SolverControl's log_history / log_result."""
        lines = []
        if depth < 2:
            return lines
        for attempt in (0, 1):
            steps, vals, res = self.solver_history(attempt)
            lines += [f"DEAL:FGMRES::Check {s}\t{v:g}" for s, v in zip(steps, vals)]
            if res:
                lines.append(f"DEAL:FGMRES::{'Convergence' if res == 1 else 'Failure'} step "
                             f"{steps[-1]} value {vals[-1]:g}")
        return lines

    def timer_summary(self):
        """TimerOutput::print_summary of the context's sections (reference names)."""
        buf = C.create_string_buffer(1 << 16)
        self._check(lib().dcp_timer_summary(self._h, buf, len(buf)))
        return buf.value.decode()

    def timer_section(self, name):
        """(calls, wall seconds) of a TimerOutput section, e.g. '   Assemble NSE system'."""
        calls, sec = C.c_long(0), C.c_double(0)
        self._check(lib().dcp_timer_section(self._h, name.encode(), C.byref(calls), C.byref(sec)))
        return calls.value, sec.value

    def set_gram_schmidt(self, kind: str):
        """DCP_OPT_GRAM_SCHMIDT of the inner Schur GMRES: "modified" (deal.II
        SolverGMRES, default), "classical2" (CGS2, device-resident cycles) or
        "dcgs2" (delayed CGS2: one reduction per Arnoldi step, device-resident)."""
        self._check(lib().dcp_set_option(self._h, OPT_GRAM_SCHMIDT,
                                         {"modified": 0, "classical2": 1, "dcgs2": 2, "sstep": 3}[kind]))

    def set_element_mfma(self, on: bool):
        """DCP_OPT_ELEMENT_MFMA: True = the velocity-block node-pair sums of the
        NSE element matrix on the matrix cores (v_mfma_f64_16x16x4_f64 Gram
        tiles) instead of FP64 VALU tiles; the same matrices up to rounding."""
        self._check(lib().dcp_set_option(self._h, OPT_ELEMENT_MFMA, int(bool(on))))

    def set_assemble_velocity_block(self, on: bool):
        """DCP_OPT_ASSEMBLE_VELOCITY_BLOCK: False (default) = assemble_nse_system
        produces nse_matrix in operator form (B^T, B, rhs, constrained-row
        diagonal; A applied matrix-free, materialised on export); True = scatter
        the velocity block too on every assembly."""
        self._check(lib().dcp_set_option(self._h, OPT_ASSEMBLE_VELOCITY_BLOCK, int(bool(on))))

    def upload_mesh(self, m: HostMesh, nse_constraints=None, T_constraints=None):
        self._feec_view = None
        nc = (nse_constraints or m.nse_constraints).as_struct()
        tc = (T_constraints or m.T_constraints).as_struct()
        self._keep = (m, nse_constraints, T_constraints)
        self._check(lib().dcp_mesh_upload(
            self._h, m.n_cells, _ptr(m.cell_nse_dofs), _ptr(m.cell_T_dofs),
            _ptr(m.cell_geometry), _ptr(m.cell_diameter), m.n_u, m.n_p, m.n_T,
            C.byref(nc), C.byref(tc)))
        self.mesh = m

    def upload_mesh_distributed(self, dm: DistMesh, comm: HostComm):
        """dcp_mesh_upload_distributed: this rank's owned + ghost cells in global
        numbering with the caller's ownership (every rank calls it)."""
        self._feec_view = None
        v = dm.as_struct()
        self._keep = (dm, v, comm)
        self._check(lib().dcp_mesh_upload_distributed(self._h, C.byref(v), C.byref(comm)))
        self.mesh = dm

    def set_state_owned(self, field, values):
        """dcp_state_set_owned: this rank's owned entries (ascending global id)."""
        a = np.ascontiguousarray(values, dtype=np.float64)
        self._check(lib().dcp_state_set_owned(self._h, field, _ptr(a), a.size))

    def get_state_owned(self, field, n):
        out = np.zeros(n)
        self._check(lib().dcp_state_get_owned(self._h, field, _ptr(out), n))
        return out

    def upload_mesh2d(self, m: HostMesh2D, nse_constraints=None, T_constraints=None):
        """dcp_mesh2d_upload: the 2D model (Standard::BoussinesqModel<2>)."""
        self._feec_view = None
        v = m.as_struct(nse_constraints, T_constraints)
        self._keep = (m, v)
        self._check(lib().dcp_mesh2d_upload(self._h, C.byref(v)))
        self.mesh = m

    # -- FEEC variant (ExteriorCalculus::BoussinesqModel<3>)
    def upload_feec_mesh(self, m: HostMesh):
        if m.feec is None:
            raise ValueError("HostMesh(feec=True) required")
        self._feec_view = m.feec.as_struct()
        self._keep = (m,)
        self._check(lib().dcp_feec_mesh_upload(self._h, C.byref(self._feec_view)))
        self.mesh = m

    def set_fgmres_max_outer(self, n: int):
        """DCP_OPT_FGMRES_MAX_OUTER (test hook): cap of the first FGMRES(30)
        (the reference's 40); lower caps force the do_solve_A fallback."""
        self._check(lib().dcp_set_option(self._h, OPT_FGMRES_MAX_OUTER, int(n)))

    def set_fused_chain(self, on: bool):
        """DCP_OPT_FUSED_CHAIN: one launch per Gram-Schmidt chain (default) or
        one per step; bitwise the same results."""
        self._check(lib().dcp_set_option(self._h, OPT_FUSED_CHAIN, int(bool(on))))

    def set_matrix_powers(self, on=True):
        """DCP_OPT_MATRIX_POWERS (default on): on several GPUs the s-step inner
        Schur GMRES exchanges each block's start vector once to S-graph depth 4
        and computes the next basis vectors on its ghost rows (bitwise the same
        iterates as one exchange per SpMV)."""
        self._check(lib().dcp_set_option(self._h, OPT_MATRIX_POWERS, int(bool(on))))

    def set_block_fixed_inner(self, k: int):
        """DCP_OPT_BLOCK_FIXED_INNER (parity hook): the block preconditioner's
        inner Schur GMRES runs exactly k steps, no tolerance test (0 = the
        reference's rule)."""
        self._check(lib().dcp_set_option(self._h, OPT_BLOCK_FIXED_INNER, int(k)))

    def set_handoff_spin_limit(self, spins: int):
        """DCP_OPT_HANDOFF_SPIN_LIMIT (test hook, process-wide): polls before a
        one-launch Gram-Schmidt hand-off counts as timed out (<= 0: default)."""
        self._check(lib().dcp_set_option(self._h, OPT_HANDOFF_SPIN_LIMIT, int(spins)))

    def set_feec_zero_mean(self, on: bool):
        self._check(lib().dcp_set_option(self._h, OPT_FEEC_ZERO_MEAN, int(bool(on))))

    def set_feec_block_preconditioner(self, on: bool):
        """DCP_OPT_FEEC_BLOCK_PRECONDITIONER (use_block_preconditioner_feec): off
        runs the identity-preconditioned GMRES(100) branch (FEEC.tpp:1420-1431)."""
        self._check(lib().dcp_set_option(self._h, OPT_FEEC_BLOCK_PRECONDITIONER, int(bool(on))))

    def set_T_fixed_cg(self, k: int):
        """DCP_OPT_T_FIXED_CG (test hook): the temperature CG runs exactly k
        steps (0 = the reference's 1e-12 |rhs| rule)."""
        self._check(lib().dcp_set_option(self._h, OPT_T_FIXED_CG, int(k)))

    def set_feec_fixed_inner(self, k: int):
        """DCP_OPT_FEEC_FIXED_INNER (test hook): both inner GMRES of the FEEC
        preconditioner run exactly k steps (0 = the reference's rule)."""
        self._check(lib().dcp_set_option(self._h, OPT_FEEC_FIXED_INNER, int(k)))

    def feec_assemble_nse_system(self):
        self._check(lib().dcp_feec_assemble_nse_system(self._h))

    def feec_build_nse_preconditioner(self):
        self._check(lib().dcp_feec_build_nse_preconditioner(self._h))

    def feec_solve_nse(self):
        it = C.c_int(0)
        rc = self._check(lib().dcp_feec_solve_nse(self._h, C.byref(it)), allow_not_converged=True)
        return rc, it.value

    def feec_cell_system(self, first, n):
        K, f = np.zeros((n, 19, 19)), np.zeros((n, 19))
        self._check(lib().dcp_feec_cell_system(self._h, first, n, _ptr(K), _ptr(f)))
        return K, f

    def feec_matrix_csr(self, which=0):
        nnz = C.c_int64(0)
        self._check(lib().dcp_feec_matrix_export(self._h, which, C.byref(nnz), None, None, None))
        n = self.mesh.feec.n
        rp, cols, vals = np.zeros(n + 1, np.int32), np.zeros(nnz.value, np.int32), np.zeros(nnz.value)
        self._check(lib().dcp_feec_matrix_export(self._h, which, C.byref(nnz), _ptr(rp), _ptr(cols),
                                                 _ptr(vals)))
        return rp, cols, vals

    # -- state
    def _size(self, field):
        m = self.mesh
        if field in (NSE_SOLUTION, OLD_NSE_SOLUTION, NSE_RHS):
            return m.feec.n if getattr(self, "_feec_view", None) is not None else m.n_u + m.n_p
        return m.n_T

    def set_state(self, field, values):
        a = np.ascontiguousarray(values, dtype=np.float64)
        self._check(lib().dcp_state_set(self._h, field, _ptr(a), a.size))

    def get_state(self, field):
        a = np.zeros(self._size(field))
        self._check(lib().dcp_state_get(self._h, field, _ptr(a), a.size))
        return a

    def copy_state(self, dst, src):
        self._check(lib().dcp_state_copy(self._h, dst, src))

    def device_ptr(self, field):
        return lib().dcp_state_device_ptr(self._h, field)

    # -- hot path
    def assemble_nse_system(self, matrix=True, rhs=True):
        flags = (ASSEMBLE_MATRIX if matrix else 0) | (ASSEMBLE_RHS if rhs else 0)
        self._check(lib().dcp_assemble_nse_system(self._h, flags))

    def build_nse_preconditioner(self):
        self._check(lib().dcp_build_nse_preconditioner(self._h))

    def assemble_temperature_matrix(self):
        self._check(lib().dcp_assemble_temperature_matrix(self._h))

    def assemble_temperature_rhs(self):
        self._check(lib().dcp_assemble_temperature_rhs(self._h))

    def solve_nse(self):
        o, i = C.c_int(0), C.c_int(0)
        rc = self._check(lib().dcp_solve_nse(self._h, C.byref(o), C.byref(i)), True)
        return rc, o.value, i.value

    def solve_nse_schur(self):
        """solve_NSE_Schur_complement: (rc, Schur GMRES steps, A^-1 solves)."""
        o, i = C.c_int(0), C.c_int(0)
        rc = self._check(lib().dcp_solve_nse_schur(self._h, C.byref(o), C.byref(i)), True)
        return rc, o.value, i.value

    def solve_temperature(self):
        it = C.c_int(0)
        rng = np.zeros(2)
        rc = self._check(lib().dcp_solve_temperature(
            self._h, C.byref(it), rng.ctypes.data_as(C.POINTER(C.c_double))), True)
        return rc, it.value, rng

    def max_velocity(self):
        v = C.c_double()
        self._check(lib().dcp_max_velocity(self._h, C.byref(v)))
        return v.value

    def cfl_number(self):
        v = C.c_double()
        self._check(lib().dcp_cfl_number(self._h, C.byref(v)))
        return v.value

    def advance_state(self):
        self._check(lib().dcp_advance_state(self._h))

    # -- exports
    def nse_matrix_csr(self):
        nnz = C.c_int64()
        self._check(lib().dcp_nse_matrix_export(self._h, C.byref(nnz), None, None, None))
        n = self.mesh.n_u + self.mesh.n_p
        rp = np.zeros(n + 1, np.int32)
        cols = np.zeros(nnz.value, np.int32)
        vals = np.zeros(nnz.value)
        self._check(lib().dcp_nse_matrix_export(self._h, C.byref(nnz), _ptr(rp), _ptr(cols),
                                                _ptr(vals)))
        return rp, cols, vals

    def T_matrix_csr(self):
        nnz = C.c_int64()
        self._check(lib().dcp_T_matrix_export(self._h, C.byref(nnz), None, None, None))
        rp = np.zeros(self.mesh.n_T + 1, np.int32)
        cols = np.zeros(nnz.value, np.int32)
        vals = np.zeros(nnz.value)
        self._check(lib().dcp_T_matrix_export(self._h, C.byref(nnz), _ptr(rp), _ptr(cols),
                                              _ptr(vals)))
        return rp, cols, vals

    def precond_diagonals(self):
        a = np.zeros(self.mesh.n_u)
        p = np.zeros(self.mesh.n_p)
        self._check(lib().dcp_precond_diagonals(self._h, _ptr(a), _ptr(p)))
        return a, p

    def cell_nse_system(self, first, n):
        dpc = 22 if getattr(self.mesh, "dim", 3) == 2 else 89
        K = np.zeros((n, dpc, dpc))
        f = np.zeros((n, dpc))
        self._check(lib().dcp_cell_nse_system(self._h, int(first), int(n), _ptr(K), _ptr(f)))
        return K, f

    def pattern_info(self) -> dict:
        v = [C.c_int64() for _ in range(5)]
        self._check(lib().dcp_pattern_info(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("nnzb_A", "nnzb_Bt", "nnzb_B", "nnz_T", "nnz_S"), (x.value for x in v)))

    def halo_selftest(self, vec, send_pos, recv_pos, n_peers: int):
        """The forward halo with self-peers: returns vec with
        vec[recv_pos] = vec[send_pos], moved through the communicator."""
        v = np.ascontiguousarray(vec, dtype=np.float64).copy()
        sp_ = np.ascontiguousarray(send_pos, dtype=np.int32)
        rp_ = np.ascontiguousarray(recv_pos, dtype=np.int32)
        self._check(lib().dcp_halo_selftest(self._h, v.size, _ptr(v), sp_.size, _ptr(sp_),
                                            _ptr(rp_), int(n_peers)))
        return v

    def scatter_info(self) -> dict:
        """Per block pattern (A, B^T, B): blocks reached by some cell's scatter
        position, the pattern size, and whether the assembly stores at first
        touch (else it zero-fills and adds)."""
        t = np.zeros(3, np.int64)
        n = np.zeros(3, np.int64)
        f = np.zeros(3, np.int32)
        self._check(lib().dcp_scatter_info(self._h, _ptr(t), _ptr(n), _ptr(f)))
        return {k: (int(t[i]), int(n[i]), bool(f[i])) for i, k in enumerate(("A", "Bt", "B"))}

    def matrix_powers_info(self) -> dict:
        """The matrix powers of the last s-step inner solve on several GPUs
        (dcp_matrix_powers_info)."""
        v = np.zeros(8, np.int64)
        self._check(lib().dcp_matrix_powers_info(self._h, _ptr(v)))
        return {"built": bool(v[0]), "n_ext": int(v[1]), "rows": [int(x) for x in v[2:5]],
                "halo_recv": int(v[5]), "value_recv": int(v[6]), "spmv_halo_recv": int(v[7])}

    def allreduce_selftest(self, vec, reps=1):
        """dcp_allreduce_selftest: vec summed over the ranks (returned), and
        the average ms of reps - 1 further back-to-back all-reduces."""
        v = np.ascontiguousarray(vec, dtype=np.float64).copy()
        ms = C.c_double(0.0)
        self._check(lib().dcp_allreduce_selftest(self._h, _ptr(v), v.size, int(reps), C.byref(ms)))
        return v, ms.value

    def comm_info(self) -> dict:
        """dcp_comm_info: the communicator as its transport reports it."""
        v = np.zeros(4, np.int32)
        self._check(lib().dcp_comm_info(self._h, _ptr(v)))
        return {"transport": {0: "none", 1: "rccl", 2: "in-process", 3: "peer"}[int(v[0])],
                "ranks": int(v[1]), "rank": int(v[2]), "device": int(v[3])}

    def local_sizes(self) -> dict:
        """dcp_local_sizes: the rank's local / owned cells and dofs."""
        v = np.zeros(8, np.int64)
        self._check(lib().dcp_local_sizes(self._h, _ptr(v)))
        keys = ("cells", "owned_cells", "n_u", "n_p", "n_T", "owned_u", "owned_p", "owned_T")
        return {k: int(x) for k, x in zip(keys, v)}

    @staticmethod
    def device_memory() -> dict:
        """dcp_device_memory: device bytes held by the buffers this host thread
        allocated (one rank's context in an in-process group), live and peak."""
        live, peak = C.c_int64(0), C.c_int64(0)
        rc = lib().dcp_device_memory(C.byref(live), C.byref(peak))
        if rc != DCP_OK:
            raise DcpError(rc, "dcp_device_memory")
        return {"live": live.value, "peak": peak.value}

    def coupling_csr(self, which: str):
        """The operator form's B^T ("Bt", 3 n_vnodes x n_p) or B ("B", n_p x n_u)
        as scalar CSR, without materialising the velocity block."""
        w = {"Bt": 0, "B": 1}[which]
        nnz = C.c_int64()
        self._check(lib().dcp_nse_coupling_export(self._h, w, C.byref(nnz), None, None, None))
        rows = self.mesh.n_u if w == 0 else self.mesh.n_p
        rp = np.zeros(rows + 1, np.int32)
        cols = np.zeros(nnz.value, np.int32)
        vals = np.zeros(nnz.value)
        self._check(lib().dcp_nse_coupling_export(self._h, w, C.byref(nnz), _ptr(rp), _ptr(cols),
                                                  _ptr(vals)))
        return rp, cols, vals

    def schur_layout(self) -> dict:
        cb, st, pm = C.c_int(), C.c_int64(), C.c_int()
        self._check(lib().dcp_schur_layout(self._h, C.byref(cb), C.byref(st), C.byref(pm)))
        return {"col_bytes": cb.value, "stored": st.value, "permuted": bool(pm.value)}

    def assembly_layout(self) -> dict:
        """dcp_assembly_layout: which forms the temperature and B^T assembly run in."""
        v = np.zeros(8, np.int64)
        self._check(lib().dcp_assembly_layout(self._h, _ptr(v)))
        return {"separable": bool(v[0]), "column_ids": int(v[1]), "layers": int(v[2]),
                "kinds": int(v[3]), "lateral_entries": int(v[4]), "bt_kronecker": bool(v[5]),
                "bt_lateral_pairs": int(v[6]), "bt_constrained_entries": int(v[7])}

    def temperature_layout(self) -> dict:
        """The temperature part of assembly_layout."""
        return self.assembly_layout()

    def timings(self) -> dict:
        t = Timings()
        self._check(lib().dcp_get_timings(self._h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in Timings._fields_}

    # -- operators on host arrays (staged through scratch device buffers)
    def _dev_roundtrip(self, fn, src, n_out):
        src = np.ascontiguousarray(src, dtype=np.float64)
        with DeviceBuffer(src.size) as d_src, DeviceBuffer(n_out) as d_dst:
            d_src.upload(src)
            rc = fn(C.c_void_p(d_src.ptr), C.c_void_p(d_dst.ptr))
            out = d_dst.download() if rc in (DCP_OK, DCP_NOT_CONVERGED) else None
        return rc, out

    def time_operator(self, which, reps, d_src, d_dst, nvec=1):
        """dcp_time_operator: ms per apply of `reps` back-to-back applies on
        device buffers (which: "nse", "velocity", "schur"), one HIP event pair;
        apply k uses vector k mod nvec of d_src / d_dst."""
        ms = C.c_double(0.0)
        w = {"nse": 0, "velocity": 1, "schur": 2}[which]
        self._check(lib().dcp_time_operator(self._h, w, int(reps), int(nvec), C.c_void_p(d_src),
                                            C.c_void_p(d_dst), C.byref(ms)))
        return ms.value

    def nse_vmult(self, src):
        n = self.mesh.n_u + self.mesh.n_p
        rc, out = self._dev_roundtrip(lambda s, d: lib().dcp_nse_vmult(self._h, s, d), src, n)
        self._check(rc)
        return out

    def run(self, rp, max_steps=0, on_step=None):
        """dcp_run: the reference's time loop from the uploaded mesh and state.
        on_step(report) is output_results' hook (return True to stop).
        Returns (rc, final report, list of per-step reports)."""
        steps = []

        def cb(_user, rep):
            r = RunReport()
            C.pointer(r)[0] = rep[0]
            steps.append(r)
            return 1 if (on_step is not None and on_step(r)) else 0

        fn = STEP_CALLBACK(cb)
        out = RunReport()
        rc = lib().dcp_run(self._h, C.byref(rp), int(max_steps), fn, None, C.byref(out))
        if rc < 0:
            self._check(rc)
        return rc, out, steps

    def velocity_vmult(self, src_u):
        """nse_matrix.block(0,0) * src_u (the do_solve_A GMRES operator)."""
        rc, out = self._dev_roundtrip(lambda s, d: lib().dcp_velocity_vmult(self._h, s, d), src_u,
                                      self.mesh.n_u)
        self._check(rc)
        return out

    def schur_vmult(self, src_p):
        rc, out = self._dev_roundtrip(lambda s, d: lib().dcp_schur_vmult(self._h, s, d), src_p,
                                      self.mesh.n_p)
        self._check(rc)
        return out

    def block_preconditioner_vmult(self, src, do_solve_A=False):
        n = self.mesh.n_u + self.mesh.n_p
        it = C.c_int(0)
        rc, out = self._dev_roundtrip(
            lambda s, d: lib().dcp_block_preconditioner_vmult(self._h, s, d, int(do_solve_A),
                                                              C.byref(it)), src, n)
        self._check(rc, True)
        return out, it.value


_hip = None


def hip() -> C.CDLL:
    """The HIP runtime libdcp.so links against (device-memory plumbing only)."""
    global _hip
    if _hip is None:
        lib()
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        _hip.hipFree.argtypes = [C.c_void_p]
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipDeviceSynchronize.argtypes = []
        _hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    return _hip


class DeviceBuffer:
    """A raw FP64 device allocation (hipMalloc) for passing d_src/d_dst pointers."""

    def __init__(self, n):
        self.n = int(n)
        p = C.c_void_p()
        rc = hip().hipMalloc(C.byref(p), max(self.n, 1) * 8)
        if rc != 0:
            raise DcpError(DCP_ERR_DEVICE, f"hipMalloc failed ({rc})")
        self.ptr = p.value
        hip().hipMemset(C.c_void_p(self.ptr), 0, max(self.n, 1) * 8)  # zero-initialised
        # the memset runs on the null stream, which the context's non-blocking
        # stream does not wait for: finish it before the buffer is handed over
        # (dst doubles as the inner solvers' initial guess, as in the reference)
        hip().hipDeviceSynchronize()

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        assert a.size == self.n
        hip().hipMemcpy(C.c_void_p(self.ptr), a.ctypes.data_as(C.c_void_p), a.nbytes, 1)

    def download(self):
        out = np.zeros(self.n)
        hip().hipDeviceSynchronize()
        hip().hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr), out.nbytes, 2)
        return out

    def close(self):
        if self.ptr:
            hip().hipFree(C.c_void_p(self.ptr))
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def physics_from_params(rp: RunParams) -> Physics:
    p = Physics()
    C.pointer(p)[0] = rp.physics
    return p


def classic_physics(time_step=0.1) -> Physics:
    """data/aqua_planet_shell_test_3d-classic.prm derived constants (L = U = 1,
    nu = 1e-2, kappa = 1e-3, beta = 0.2, T_ref = 2, g = 1)."""
    return Physics(time_step, 1.0 / 100.0, 1.0 / 1000.0, 0.2, 2.0, 1.0, 1.0, 1.0, 1.0, 0, 1, 1)
