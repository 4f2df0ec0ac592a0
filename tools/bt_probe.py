"""Is the assembled B^T block bitwise the transpose of the B block? (GPU)"""
import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT","/root/repo"), "3d-dycoreplanet_amd"))
import numpy as np, scipy.sparse as sp, dcp
for R in (2, 3):
    m = dcp.HostMesh(refine=R)
    ctx = dcp.Context(device=0)
    ctx.set_physics(dcp.classic_physics())
    ctx.upload_mesh(m)
    rng = np.random.default_rng(5)
    ctx.set_state(dcp.OLD_NSE_SOLUTION, rng.uniform(-1, 1, m.n_u + m.n_p))
    ctx.set_state(dcp.OLD_T_SOLUTION, m.T0)
    ctx.assemble_nse_system()
    n = m.n_u + m.n_p
    rp, cols, vals = ctx.nse_matrix_csr()
    A = sp.csr_matrix((vals, cols, rp), shape=(n, n))
    Bt = A[:m.n_u, m.n_u:].tocsr(); B = A[m.n_u:, :m.n_u].tocsr()
    D = (Bt - B.T.tocsr())
    D.eliminate_zeros()
    print(R, "nnz Bt", Bt.nnz, "nnz B", B.nnz, "differing entries", D.nnz, "max", abs(D).max() if D.nnz else 0.0, flush=True)
    ctx.close()
