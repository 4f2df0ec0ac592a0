// output_results (include/core/boussinesq_model.tpp:1566-1680) for the classic
// model: the joint [u p T] solution through DataOut::build_patches(
// nse_velocity_degree = 2) and write_vtu / write_pvtu_record.
//
// One patch per cell: the (2+1)^3 lattice of reference points {0, 1/2, 1}^3,
// placed by DataOut's default MappingQ1 (the trilinear map of the cell's 8
// vertices = the corner support points of its MappingQ(3) data), 2^3
// sub-hexahedra; point data of the Postprocessor (:1492-1554): "velocity"
// (the Q2 nodal values, which the lattice points are), "p" and "T" (Q1,
// trilinear), "partition". Written as VTU XML with ASCII data arrays (deal.II
// compresses with zlib when it has it; the arrays and topology are the same).
// Host-only: reads global solution vectors (dcp_state_get).
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/dcp.h"
#include "fe_tables.h"

namespace {

struct LocalMaps {
  int vel[27][3];  // lexicographic Q2 node, component -> FESystem local dof
  int pre[8];      // vertex -> local dof
  LocalMaps() {
    for (int i = 0; i < dcp::kNseDofs; ++i) {
      const dcp::SysDof s = dcp::system_dof(i);
      if (s.comp < 3) vel[s.lex][s.comp] = i;
      else pre[s.lex] = i;
    }
  }
};

double trilinear(const double v[8], double x, double y, double z) {
  return (1 - z) * ((1 - y) * ((1 - x) * v[0] + x * v[1]) + y * ((1 - x) * v[2] + x * v[3])) +
         z * ((1 - y) * ((1 - x) * v[4] + x * v[5]) + y * ((1 - x) * v[6] + x * v[7]));
}

}  // namespace

extern "C" int dcp_write_vtu(const dcp_host_mesh_view* m, const double* nse, const double* T,
                             int partition, const char* path) {
  if (!m || !nse || !T || !path || m->n_cells <= 0) return DCP_ERR_INVALID;
  FILE* f = std::fopen(path, "w");
  if (!f) return DCP_ERR_INVALID;
  static const LocalMaps maps;
  const long nc = m->n_cells, np = 27 * nc, nh = 8 * nc;
  std::fprintf(f,
               "<?xml version=\"1.0\" ?>\n<!-- output_results: DataOut::build_patches(2), "
               "libdcp -->\n<VTKFile type=\"UnstructuredGrid\" version=\"0.1\" "
               "byte_order=\"LittleEndian\">\n<UnstructuredGrid>\n"
               "<Piece NumberOfPoints=\"%ld\" NumberOfCells=\"%ld\">\n"
               "  <Points>\n    <DataArray type=\"Float64\" NumberOfComponents=\"3\" "
               "format=\"ascii\">\n",
               np, nh);
  auto vertex = [&](long c, int v, int d) {
    const int a = 3 * (v & 1), b = 3 * ((v >> 1) & 1), cc = 3 * (v >> 2);
    return m->cell_geometry[(64 * c + a + 4 * b + 16 * cc) * 3 + d];
  };
  for (long c = 0; c < nc; ++c)
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) {
          double xv[3];
          for (int d = 0; d < 3; ++d) {
            double vv[8];
            for (int v = 0; v < 8; ++v) vv[v] = vertex(c, v, d);
            xv[d] = trilinear(vv, 0.5 * i, 0.5 * j, 0.5 * k);
          }
          std::fprintf(f, "%.17g %.17g %.17g\n", xv[0], xv[1], xv[2]);
        }
  std::fprintf(f, "    </DataArray>\n  </Points>\n  <Cells>\n"
                  "    <DataArray type=\"Int64\" Name=\"connectivity\" format=\"ascii\">\n");
  for (long c = 0; c < nc; ++c)
    for (int kz = 0; kz < 2; ++kz)
      for (int jy = 0; jy < 2; ++jy)
        for (int ix = 0; ix < 2; ++ix) {
          auto id = [&](int i, int j, int k) { return 27 * c + i + 3 * j + 9 * k; };
          // VTK_HEXAHEDRON: bottom face counter-clockwise, then the top face
          std::fprintf(f, "%ld %ld %ld %ld %ld %ld %ld %ld\n", id(ix, jy, kz), id(ix + 1, jy, kz),
                       id(ix + 1, jy + 1, kz), id(ix, jy + 1, kz), id(ix, jy, kz + 1),
                       id(ix + 1, jy, kz + 1), id(ix + 1, jy + 1, kz + 1), id(ix, jy + 1, kz + 1));
        }
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"Int64\" Name=\"offsets\" format=\"ascii\">\n");
  for (long h = 1; h <= nh; ++h) std::fprintf(f, "%ld\n", 8 * h);
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"UInt8\" Name=\"types\" format=\"ascii\">\n");
  for (long h = 0; h < nh; ++h) std::fprintf(f, "12\n");
  std::fprintf(f, "    </DataArray>\n  </Cells>\n  <PointData Scalars=\"p\" Vectors=\"velocity\">\n"
                  "    <DataArray type=\"Float64\" Name=\"velocity\" NumberOfComponents=\"3\" "
                  "format=\"ascii\">\n");
  for (long c = 0; c < nc; ++c) {
    const int32_t* d = m->cell_nse_dofs + 89 * c;
    for (int l = 0; l < 27; ++l)
      std::fprintf(f, "%.17g %.17g %.17g\n", nse[d[maps.vel[l][0]]], nse[d[maps.vel[l][1]]],
                   nse[d[maps.vel[l][2]]]);
  }
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"Float64\" Name=\"p\" format=\"ascii\">\n");
  for (long c = 0; c < nc; ++c) {
    const int32_t* d = m->cell_nse_dofs + 89 * c;
    double pv[8];
    for (int v = 0; v < 8; ++v) pv[v] = nse[d[maps.pre[v]]];
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i)
          std::fprintf(f, "%.17g\n", trilinear(pv, 0.5 * i, 0.5 * j, 0.5 * k));
  }
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"Float64\" Name=\"T\" format=\"ascii\">\n");
  for (long c = 0; c < nc; ++c) {
    double tv[8];
    for (int v = 0; v < 8; ++v) tv[v] = T[m->cell_T_dofs[8 * c + v]];
    for (int k = 0; k < 3; ++k)
      for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i)
          std::fprintf(f, "%.17g\n", trilinear(tv, 0.5 * i, 0.5 * j, 0.5 * k));
  }
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"Float64\" Name=\"partition\" "
                  "format=\"ascii\">\n");
  for (long p = 0; p < np; ++p) std::fprintf(f, "%d\n", partition);
  std::fprintf(f, "    </DataArray>\n  </PointData>\n</Piece>\n</UnstructuredGrid>\n</VTKFile>\n");
  const bool ok = std::ferror(f) == 0;
  std::fclose(f);
  return ok ? DCP_OK : DCP_ERR_INVALID;
}

namespace {
int write_pvtu(const char* path, int n_pieces, const char* const* pieces, bool vorticity) {
  if (!path || n_pieces <= 0 || !pieces) return DCP_ERR_INVALID;
  FILE* f = std::fopen(path, "w");
  if (!f) return DCP_ERR_INVALID;
  std::fprintf(f, "<?xml version=\"1.0\"?>\n<VTKFile type=\"PUnstructuredGrid\" version=\"0.1\" "
                  "byte_order=\"LittleEndian\">\n  <PUnstructuredGrid GhostLevel=\"0\">\n"
                  "    <PPointData Scalars=\"p\" Vectors=\"velocity\">\n");
  if (vorticity)
    std::fprintf(f, "      <PDataArray type=\"Float64\" Name=\"vorticity\" NumberOfComponents=\"3\" "
                    "format=\"ascii\"/>\n");
  std::fprintf(f, "      <PDataArray type=\"Float64\" Name=\"velocity\" NumberOfComponents=\"3\" "
                  "format=\"ascii\"/>\n"
                  "      <PDataArray type=\"Float64\" Name=\"p\" format=\"ascii\"/>\n"
                  "      <PDataArray type=\"Float64\" Name=\"T\" format=\"ascii\"/>\n"
                  "      <PDataArray type=\"Float64\" Name=\"partition\" format=\"ascii\"/>\n"
                  "    </PPointData>\n    <PPoints>\n"
                  "      <PDataArray type=\"Float64\" NumberOfComponents=\"3\"/>\n"
                  "    </PPoints>\n");
  for (int i = 0; i < n_pieces; ++i)
    std::fprintf(f, "    <Piece Source=\"%s\"/>\n", pieces[i]);
  std::fprintf(f, "  </PUnstructuredGrid>\n</VTKFile>\n");
  const bool ok = std::ferror(f) == 0;
  std::fclose(f);
  return ok ? DCP_OK : DCP_ERR_INVALID;
}
}  // namespace

extern "C" int dcp_write_pvtu_record(const char* path, int n_pieces, const char* const* pieces) {
  return write_pvtu(path, n_pieces, pieces, false);
}

extern "C" int dcp_write_feec_pvtu_record(const char* path, int n_pieces,
                                          const char* const* pieces) {
  return write_pvtu(path, n_pieces, pieces, true);
}

// ---------------------------------------------------------------------------
// output_results of the FEEC model (boussineq_model_FEEC.tpp:1917-2030 with
// the Postprocessor of :1808-1912): the joint [w u p T] solution through
// DataOut::build_patches(min(nse_velocity_degree, temperature_degree) = 1), so
// one patch per cell = the cell itself (its 8 vertices, one hexahedron),
// point data "vorticity" (Nedelec(0), covariant Piola), "velocity" (RT(0),
// contravariant Piola), "p" (DGQ0), "T" (Q1), "partition", evaluated at the
// vertices with the cell's MappingQ1. The Nedelec / RT local functions carry
// the library's global orientation signs (FEEC conventions), the
// same basis the FEEC kernels assemble with.
namespace {

inline double lin01(int s, double t) { return s ? t : 1.0 - t; }
inline double dlin01(int s) { return s ? 1.0 : -1.0; }
// deal.II line order: (axis, transverse b, transverse c, side on b, side on c)
constexpr int kFeecLine[12][5] = {{1, 0, 2, 0, 0}, {1, 0, 2, 1, 0}, {0, 1, 2, 0, 0},
                                  {0, 1, 2, 1, 0}, {1, 0, 2, 0, 1}, {1, 0, 2, 1, 1},
                                  {0, 1, 2, 0, 1}, {0, 1, 2, 1, 1}, {2, 0, 1, 0, 0},
                                  {2, 0, 1, 1, 0}, {2, 0, 1, 0, 1}, {2, 0, 1, 1, 1}};

// w, u at reference point xi of cell c (MappingQ1 of its 8 vertices)
void feec_fields(const dcp_feec_mesh* m, const double* nse, long c, const double xi[3],
                 double w[3], double u[3]) {
  const double* X = m->cell_vertices + 24 * c;
  double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  for (int v = 0; v < 8; ++v) {
    const int a = v & 1, b = (v >> 1) & 1, cc = v >> 2;
    const double la = lin01(a, xi[0]), lb = lin01(b, xi[1]), lc = lin01(cc, xi[2]);
    const double d[3] = {dlin01(a) * lb * lc, la * dlin01(b) * lc, la * lb * dlin01(cc)};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) J[i][j] += X[3 * v + i] * d[j];
  }
  const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
  const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
  const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
  const double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
  // rows of J^-1 (Ji[a][i]): (J^-T N)_i = Ji[a][i] g for N = g e_a
  double Ji[3][3];
  Ji[0][0] = c00 / det;
  Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
  Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
  Ji[1][0] = c01 / det;
  Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
  Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
  Ji[2][0] = c02 / det;
  Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
  Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
  for (int i = 0; i < 3; ++i) w[i] = u[i] = 0.0;
  for (int l = 0; l < 12; ++l) {
    const int a = kFeecLine[l][0], b = kFeecLine[l][1], cc = kFeecLine[l][2];
    const double g = lin01(kFeecLine[l][3], xi[b]) * lin01(kFeecLine[l][4], xi[cc]);
    const double coef = m->sign_w[12 * c + l] * nse[m->cell_w[12 * c + l]];
    for (int i = 0; i < 3; ++i) w[i] += coef * Ji[a][i] * g;
  }
  for (int f = 0; f < 6; ++f) {
    const int a = f / 2;
    const double r = lin01(f % 2, xi[a]);
    const double coef = m->sign_u[6 * c + f] * nse[m->n_w + m->cell_u[6 * c + f]];
    for (int i = 0; i < 3; ++i) u[i] += coef * J[i][a] * r / det;
  }
}

}  // namespace

extern "C" int dcp_write_feec_vtu(const dcp_feec_mesh* m, const double* nse, const double* T,
                                  int partition, const char* path) {
  if (!m || !nse || !T || !path || m->n_cells <= 0) return DCP_ERR_INVALID;
  FILE* f = std::fopen(path, "w");
  if (!f) return DCP_ERR_INVALID;
  const long nc = m->n_cells, np = 8 * nc;
  std::fprintf(f,
               "<?xml version=\"1.0\" ?>\n<!-- output_results (FEEC): DataOut::build_patches(1), "
               "libdcp -->\n<VTKFile type=\"UnstructuredGrid\" version=\"0.1\" "
               "byte_order=\"LittleEndian\">\n<UnstructuredGrid>\n"
               "<Piece NumberOfPoints=\"%ld\" NumberOfCells=\"%ld\">\n"
               "  <Points>\n    <DataArray type=\"Float64\" NumberOfComponents=\"3\" "
               "format=\"ascii\">\n",
               np, nc);
  for (long p = 0; p < np; ++p) {
    const double* x = m->cell_vertices + 3 * p;
    std::fprintf(f, "%.17g %.17g %.17g\n", x[0], x[1], x[2]);
  }
  std::fprintf(f, "    </DataArray>\n  </Points>\n  <Cells>\n"
                  "    <DataArray type=\"Int64\" Name=\"connectivity\" format=\"ascii\">\n");
  for (long c = 0; c < nc; ++c) {
    const long b = 8 * c;  // lexicographic vertices -> VTK_HEXAHEDRON order
    std::fprintf(f, "%ld %ld %ld %ld %ld %ld %ld %ld\n", b, b + 1, b + 3, b + 2, b + 4, b + 5, b + 7,
                 b + 6);
  }
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"Int64\" Name=\"offsets\" format=\"ascii\">\n");
  for (long h = 1; h <= nc; ++h) std::fprintf(f, "%ld\n", 8 * h);
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"UInt8\" Name=\"types\" format=\"ascii\">\n");
  for (long h = 0; h < nc; ++h) std::fprintf(f, "12\n");
  std::fprintf(f, "    </DataArray>\n  </Cells>\n  <PointData Scalars=\"p\" Vectors=\"velocity\">\n");
  std::vector<double> W(3 * np), U(3 * np);
  for (long c = 0; c < nc; ++c)
    for (int v = 0; v < 8; ++v) {
      const double xi[3] = {double(v & 1), double((v >> 1) & 1), double(v >> 2)};
      feec_fields(m, nse, c, xi, &W[3 * (8 * c + v)], &U[3 * (8 * c + v)]);
    }
  for (int fld = 0; fld < 2; ++fld) {
    std::fprintf(f, "    <DataArray type=\"Float64\" Name=\"%s\" NumberOfComponents=\"3\" "
                    "format=\"ascii\">\n", fld == 0 ? "vorticity" : "velocity");
    const std::vector<double>& V = fld == 0 ? W : U;
    for (long p = 0; p < np; ++p)
      std::fprintf(f, "%.17g %.17g %.17g\n", V[3 * p], V[3 * p + 1], V[3 * p + 2]);
    std::fprintf(f, "    </DataArray>\n");
  }
  std::fprintf(f, "    <DataArray type=\"Float64\" Name=\"p\" format=\"ascii\">\n");
  for (long c = 0; c < nc; ++c)
    for (int v = 0; v < 8; ++v) std::fprintf(f, "%.17g\n", nse[m->n_w + m->n_u + c]);
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"Float64\" Name=\"T\" format=\"ascii\">\n");
  for (long p = 0; p < np; ++p) std::fprintf(f, "%.17g\n", T[m->cell_T_dofs[p]]);
  std::fprintf(f, "    </DataArray>\n    <DataArray type=\"Float64\" Name=\"partition\" "
                  "format=\"ascii\">\n");
  for (long p = 0; p < np; ++p) std::fprintf(f, "%d\n", partition);
  std::fprintf(f, "    </DataArray>\n  </PointData>\n</Piece>\n</UnstructuredGrid>\n</VTKFile>\n");
  const bool ok = std::ferror(f) == 0;
  std::fclose(f);
  return ok ? DCP_OK : DCP_ERR_INVALID;
}
