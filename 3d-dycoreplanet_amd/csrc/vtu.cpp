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

extern "C" int dcp_write_pvtu_record(const char* path, int n_pieces, const char* const* pieces) {
  if (!path || n_pieces <= 0 || !pieces) return DCP_ERR_INVALID;
  FILE* f = std::fopen(path, "w");
  if (!f) return DCP_ERR_INVALID;
  std::fprintf(f, "<?xml version=\"1.0\"?>\n<VTKFile type=\"PUnstructuredGrid\" version=\"0.1\" "
                  "byte_order=\"LittleEndian\">\n  <PUnstructuredGrid GhostLevel=\"0\">\n"
                  "    <PPointData Scalars=\"p\" Vectors=\"velocity\">\n"
                  "      <PDataArray type=\"Float64\" Name=\"velocity\" NumberOfComponents=\"3\" "
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
