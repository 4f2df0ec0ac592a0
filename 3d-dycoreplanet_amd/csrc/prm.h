// .prm configuration layer: a native restatement of the reference's three
// ParameterHandler consumers (no deal.II).
//
//   CoreModelData::Parameters          source/model_data/boussinesq_model_parameters.cc:6-48,52-185,189-239
//   CoreModelData::PhysicalConstants   source/model_data/physical_constants.cc:6-46,50-131,135-167
//   CoreModelData::ReferenceQuantities source/model_data/reference_quantities.cc:6-33,37-67,71-88
//
// Each of the three reads the same file independently with skip_undefined =
// true; here one tokenizer reads the file once into "path/key" -> value and
// each struct pulls only its declared entries (declared defaults win over the
// reference constructors' member-initialiser defaults, Appendix A Q13).
#pragma once
#include <map>
#include <stdexcept>
#include <string>

namespace dcp {

struct PrmError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Flat view of a deal.II ParameterHandler text file.
class PrmFile {
 public:
  // Parses `text` (subsection/end/set/# comment grammar). Throws PrmError on
  // malformed input (unbalanced subsection/end, set without '=').
  static PrmFile parse(const std::string& text);
  // Reads a file; missing file -> PrmError (the caller decides whether to emit
  // a template, reference behaviour boussinesq_model_parameters.cc:32-42).
  static PrmFile read(const std::string& filename);

  bool has(const std::string& path) const { return kv_.count(path) != 0; }
  // Returns value or `def` when the entry is absent (skip_undefined semantics).
  std::string get(const std::string& path, const std::string& def) const;
  double get_double(const std::string& path, const std::string& def) const;
  long get_integer(const std::string& path, const std::string& def) const;
  bool get_bool(const std::string& path, const std::string& def) const;
  const std::map<std::string, std::string>& entries() const { return kv_; }

 private:
  std::map<std::string, std::string> kv_;
};

// reference_quantities.cc:71-88
struct ReferenceQuantities {
  double time = 0;
  double velocity = 10;
  double length = 1e+4;
  double temperature_ref = 273.15;
  double temperature_change = 5;
  void parse(const PrmFile& f);
};

// physical_constants.cc:135-167 (nu = mu/rho :150, kappa = k/(c_p p) :156, R1 = R0 + h :164)
struct PhysicalConstants {
  double pressure = 1.01325e+5;
  double omega = 7.272205e-5;
  double density = 1.29;
  double universal_gas_constant = 8.31446261815324;
  double specific_gas_constant_dry = 287.0;
  double expansion_coefficient = 0.003661;
  double dynamic_viscosity = 1.82e-5;
  double kinematic_viscosity = 0;
  double specific_heat_p = 1.005;
  double specific_heat_v = 0.718;
  double thermal_conductivity = 2.62e-2;
  double thermal_diffusivity = 0;
  double radiogenic_heating = 7.4e-12;
  double gravity_constant = 9.81;
  double speed_of_sound = 331.5;
  double atm_height = 1.0e+5;
  double R0 = 6.371000e+6;
  double R1 = 0;
  void parse(const PrmFile& f);
};

// boussinesq_model_parameters.cc:189-239
struct Parameters {
  unsigned space_dimension = 2;
  ReferenceQuantities reference_quantities;
  PhysicalConstants physical_constants;
  double final_time = 1.0;
  double time_step = 0.1;
  bool adapt_time_step = false;
  unsigned initial_global_refinement = 3;
  bool cuboid_geometry = false;
  double nse_theta = 0.5;
  unsigned nse_velocity_degree = 2;
  bool use_FEEC_solver = false;
  bool use_block_preconditioner_feec = true;
  bool correct_pressure_to_zero_mean = false;
  bool use_locally_conservative_discretization = true;
  unsigned solver_diagnostics_print_level = 1;
  bool use_schur_complement_solver = false;
  bool use_direct_solver = false;
  unsigned NSE_solver_interval = 1;
  double temperature_theta = 0.5;
  unsigned temperature_degree = 2;
  std::string filename_output = "dycore";
  std::string dirname_output = "data-output";
  bool hello_from_cluster = false;

  void parse(const PrmFile& f);
  // Reference constructor semantics: read file; if it is missing, write a
  // template with the declared defaults to that path and throw.
  static Parameters from_file(const std::string& filename);
  // Template text with every declared entry at its declared default.
  static std::string template_text();

  // Derived non-dimensional numbers (core_model_data.cc:7-22).
  double reynolds() const;
  double peclet() const;
};

}  // namespace dcp
