// Reference-cell data shared by the host setup code and the HIP kernels:
// local numbering of the Q2 / Q1 Lagrange elements and of the Taylor-Hood
// system element, and the 3-point Gauss rule.
//
// Numbering follows deal.II's conventions that the reference relies on
// through FESystem(FE_Q(2)^3, FE_Q(1)) (boussinesq_model.tpp:21-28) and
// QGauss(deg+1) (boussinesq_model.tpp:708):
//   * vertices v = i + 2j + 4k, lines 0..11, faces 0..5 (x0,x1,y0,y1,z0,z1),
//     interior; FE_Q(2) hierarchic order = vertices, lines, faces, interior;
//   * FESystem interleaves per geometric object: 4 dofs per vertex
//     (u_x,u_y,u_z,p), then 3 per line, 3 per face, 3 interior = 89;
//   * QGauss(n): tensor product, x fastest.
// Internally all kernels use LEXICOGRAPHIC node order (a + 3b + 9c over the
// 1D points {0, 1/2, 1}); kQ2HierToLex maps a hierarchic index to it.
#pragma once

namespace dcp {

constexpr int kQ2 = 27;         // scalar Q2 nodes per hex
constexpr int kQ1 = 8;          // scalar Q1 nodes per hex
constexpr int kNseDofs = 89;    // 3*27 + 8
constexpr int kNQ = 27;         // QGauss(3) points per hex

// Hierarchic FE_Q(2) index -> lexicographic (a + 3b + 9c) position.
constexpr int kQ2HierToLex[27] = {
    // vertices 0..7: (2i,2j,2k)
    0, 2, 6, 8, 18, 20, 24, 26,
    // lines 0..11
    3,   // line 0: x=0,z=0 along y -> (0,1,0)
    5,   // line 1: x=1,z=0         -> (2,1,0)
    1,   // line 2: y=0,z=0 along x -> (1,0,0)
    7,   // line 3: y=1,z=0         -> (1,2,0)
    21,  // line 4: x=0,z=1         -> (0,1,2)
    23,  // line 5: x=1,z=1         -> (2,1,2)
    19,  // line 6: y=0,z=1         -> (1,0,2)
    25,  // line 7: y=1,z=1         -> (1,2,2)
    9,   // line 8: x=0,y=0 along z -> (0,0,1)
    11,  // line 9: x=1,y=0         -> (2,0,1)
    15,  // line 10: x=0,y=1        -> (0,2,1)
    17,  // line 11: x=1,y=1        -> (2,2,1)
    // faces 0..5
    12,  // x=0 -> (0,1,1)
    14,  // x=1 -> (2,1,1)
    10,  // y=0 -> (1,0,1)
    16,  // y=1 -> (1,2,1)
    4,   // z=0 -> (1,1,0)
    22,  // z=1 -> (1,1,2)
    // interior
    13};

// Lexicographic position of Q1 vertex v (deal.II vertex order is lexicographic).
constexpr int kQ1VertexToQ2Lex[8] = {0, 2, 6, 8, 18, 20, 24, 26};

// FESystem local dof -> (component, lexicographic scalar index).
// component 0..2 = velocity, 3 = pressure (scalar index is then the vertex 0..7).
struct SysDof {
  int comp;
  int lex;
};

constexpr SysDof system_dof(int i) {
  // vertices: 4 per vertex
  return i < 32 ? SysDof{i % 4, i % 4 == 3 ? i / 4 : kQ2HierToLex[i / 4]}
                : SysDof{(i - 32) % 3, kQ2HierToLex[8 + (i - 32) / 3]};
}

// 1D Gauss-Legendre 3-point rule on [0,1].
constexpr double kGaussX[3] = {0.11270166537925831148, 0.5, 0.88729833462074168852};
constexpr double kGaussW[3] = {0.27777777777777777778, 0.44444444444444444444,
                               0.27777777777777777778};

// Cell geometry = MappingQ(3) (boussinesq_model.tpp:20, `const MappingQ<dim>
// mapping` at boussinesq_model.h:211): MappingQGeneric's tensor-product
// Lagrange basis on the 4 Gauss-Lobatto points of [0,1], i.e. 64 support
// points per cell in lexicographic order (i + 4j + 16k). A cell the reference
// maps with MappingQ1 (deal.II 9.2: cells without boundary lines) is passed as
// the trilinear interpolant at those 64 points, which the cubic basis
// reproduces exactly.
constexpr int kMapPts1 = 4;
constexpr int kMapPts = 64;
constexpr double kGL3[4] = {0.0, 0.27639320225002103036, 0.72360679774997896964, 1.0};

constexpr double map_lag(int i, double x) {
  double v = 1.0;
  for (int j = 0; j < 4; ++j)
    if (j != i) v *= (x - kGL3[j]) / (kGL3[i] - kGL3[j]);
  return v;
}
constexpr double map_dlag(int i, double x) {
  double s = 0.0;
  for (int k = 0; k < 4; ++k) {
    if (k == i) continue;
    double v = 1.0 / (kGL3[i] - kGL3[k]);
    for (int j = 0; j < 4; ++j)
      if (j != i && j != k) v *= (x - kGL3[j]) / (kGL3[i] - kGL3[j]);
    s += v;
  }
  return s;
}

}  // namespace dcp
