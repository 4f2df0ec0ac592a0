// .prm parser + parameter structs. See prm.h for the reference citations.
#include "prm.h"

#include <cctype>
#include <cmath>
#include <iterator>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <vector>

namespace dcp {

namespace {

std::string trim(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

// Collapse runs of whitespace into one blank (keys such as
// "initial  global refinement" name the same entry).
std::string normalize(const std::string& s) {
  std::string out;
  bool blank = false;
  for (char c : trim(s)) {
    if (std::isspace(static_cast<unsigned char>(c))) {
      blank = true;
    } else {
      if (blank && !out.empty()) out.push_back(' ');
      blank = false;
      out.push_back(c);
    }
  }
  return out;
}

std::string strip_comment(const std::string& line) {
  std::string out;
  for (size_t i = 0; i < line.size(); ++i) {
    if (line[i] == '\\' && i + 1 < line.size() && line[i + 1] == '#') {
      out.push_back('#');
      ++i;
    } else if (line[i] == '#') {
      break;
    } else {
      out.push_back(line[i]);
    }
  }
  return out;
}

bool starts_with_word(const std::string& s, const char* w) {
  const size_t n = std::char_traits<char>::length(w);
  return s.size() >= n && s.compare(0, n, w) == 0 &&
         (s.size() == n || std::isspace(static_cast<unsigned char>(s[n])));
}

}  // namespace

PrmFile PrmFile::parse(const std::string& text) {
  PrmFile f;
  std::vector<std::string> stack;
  std::istringstream in(text);
  std::string raw, line;
  int lineno = 0;
  while (std::getline(in, raw)) {
    ++lineno;
    // deal.II joins lines ending in a backslash.
    while (!raw.empty() && raw.back() == '\\') {
      std::string next;
      raw.pop_back();
      if (!std::getline(in, next)) break;
      ++lineno;
      raw += " " + next;
    }
    line = trim(strip_comment(raw));
    if (line.empty()) continue;
    if (starts_with_word(line, "subsection")) {
      stack.push_back(normalize(line.substr(10)));
    } else if (line == "end") {
      if (stack.empty())
        throw PrmError("prm line " + std::to_string(lineno) + ": 'end' without subsection");
      stack.pop_back();
    } else if (starts_with_word(line, "set")) {
      const std::string rest = line.substr(3);
      const size_t eq = rest.find('=');
      if (eq == std::string::npos)
        throw PrmError("prm line " + std::to_string(lineno) + ": 'set' without '='");
      std::string path;
      for (const auto& s : stack) path += s + "/";
      path += normalize(rest.substr(0, eq));
      f.kv_[path] = trim(rest.substr(eq + 1));
    } else if (starts_with_word(line, "include") || starts_with_word(line, "alias")) {
      // Not used by any reference .prm; treated as undefined and skipped.
    } else {
      throw PrmError("prm line " + std::to_string(lineno) + ": cannot parse '" + line + "'");
    }
  }
  if (!stack.empty()) throw PrmError("prm: unterminated subsection '" + stack.back() + "'");
  return f;
}

PrmFile PrmFile::read(const std::string& filename) {
  std::ifstream in(filename);
  if (!in) throw PrmError("Input parameter file <" + filename + "> not found.");
  std::stringstream ss;
  ss << in.rdbuf();
  return parse(ss.str());
}

std::string PrmFile::get(const std::string& path, const std::string& def) const {
  auto it = kv_.find(path);
  return it == kv_.end() ? def : it->second;
}

double PrmFile::get_double(const std::string& path, const std::string& def) const {
  const std::string s = get(path, def);
  char* end = nullptr;
  const double v = std::strtod(s.c_str(), &end);
  if (end == s.c_str() || trim(end).size() != 0)
    throw PrmError("entry <" + path + "> = '" + s + "' is not a double");
  return v;
}

long PrmFile::get_integer(const std::string& path, const std::string& def) const {
  const std::string s = get(path, def);
  char* end = nullptr;
  const long v = std::strtol(s.c_str(), &end, 10);
  if (end == s.c_str() || trim(end).size() != 0)
    throw PrmError("entry <" + path + "> = '" + s + "' is not an integer");
  return v;
}

bool PrmFile::get_bool(const std::string& path, const std::string& def) const {
  const std::string s = get(path, def);
  if (s == "true" || s == "yes") return true;
  if (s == "false" || s == "no") return false;
  throw PrmError("entry <" + path + "> = '" + s + "' is not a bool");
}

// ---------------------------------------------------------------------------
// Declared entries (path, default). The defaults are the *declared* defaults
// of declare_parameters(), which are what a parse without the entry yields.
namespace {
struct Decl {
  const char* path;
  const char* def;
};
const Decl kReferenceQuantities[] = {
    // reference_quantities.cc:37-67
    {"Boussinesq Model/Reference quantities/velocity", "10"},
    {"Boussinesq Model/Reference quantities/length", "1e+4"},
    {"Boussinesq Model/Reference quantities/temperature", "273.15"},
    {"Boussinesq Model/Reference quantities/temperature change", "5"},
};
const Decl kPhysicalConstants[] = {
    // physical_constants.cc:50-131
    {"Physical Constants/omega", "7.272205e-5"},
    {"Physical Constants/average atm pressure", "1.01325e+5"},
    {"Physical Constants/density", "1.29"},
    {"Physical Constants/universal gas constant", "8.31446261815324"},
    {"Physical Constants/specific gas constant dry", "287.0"},
    {"Physical Constants/expansion coefficient", "0.003661"},
    {"Physical Constants/dynamic viscosity", "1.82e-5"},
    {"Physical Constants/specific heat p", "1.005"},
    {"Physical Constants/specific heat v", "0.718"},
    {"Physical Constants/thermal conductivity", "2.62e-2"},
    {"Physical Constants/radiogenic heating", "7.4e-12"},
    {"Physical Constants/gravity constant", "9.81"},
    {"Physical Constants/speed of sound", "331.5"},
    {"Physical Constants/atm height", "1.0e+5"},
    {"Physical Constants/R0", "6.371000e+6"},
};
const Decl kParameters[] = {
    // boussinesq_model_parameters.cc:52-185
    {"Boussinesq Model/Mesh parameters/initial global refinement", "3"},
    {"Boussinesq Model/Mesh parameters/cuboid geometry", "false"},
    {"Boussinesq Model/space dimension", "2"},
    {"Boussinesq Model/final time", "1.0"},
    {"Boussinesq Model/time step", "0.1"},
    {"Boussinesq Model/adapt time step", "false"},
    {"Boussinesq Model/nse theta", "0.5"},
    {"Boussinesq Model/nse velocity degree", "2"},
    {"Boussinesq Model/use FEEC solver", "false"},
    {"Boussinesq Model/use block preconditioner feec", "true"},
    {"Boussinesq Model/correct pressure to zero mean", "false"},
    {"Boussinesq Model/use locally conservative discretization", "true"},
    {"Boussinesq Model/solver diagnostics level", "1"},
    {"Boussinesq Model/use schur complement solver", "false"},
    {"Boussinesq Model/use direct solver", "false"},
    {"Boussinesq Model/NSE solver interval", "1"},
    {"Boussinesq Model/temperature theta", "0.5"},
    {"Boussinesq Model/temperature degree", "2"},
    {"Boussinesq Model/filename output", "dycore"},
    {"Boussinesq Model/dirname output", "data-output"},
    {"Boussinesq Model/hello from cluster", "false"},
};

template <size_t N>
const char* def_of(const Decl (&tab)[N], const char* path) {
  for (const auto& d : tab)
    if (std::string(d.path) == path) return d.def;
  throw PrmError(std::string("internal: undeclared entry ") + path);
}
}  // namespace

void ReferenceQuantities::parse(const PrmFile& f) {
  auto D = [&](const char* p) { return f.get_double(p, def_of(kReferenceQuantities, p)); };
  velocity = D("Boussinesq Model/Reference quantities/velocity");
  length = D("Boussinesq Model/Reference quantities/length");
  temperature_ref = D("Boussinesq Model/Reference quantities/temperature");
  temperature_change = D("Boussinesq Model/Reference quantities/temperature change");
  time = length / velocity;  // reference_quantities.cc:87
}

void PhysicalConstants::parse(const PrmFile& f) {
  auto D = [&](const char* p) { return f.get_double(p, def_of(kPhysicalConstants, p)); };
  pressure = D("Physical Constants/average atm pressure");
  omega = D("Physical Constants/omega");
  density = D("Physical Constants/density");
  universal_gas_constant = D("Physical Constants/universal gas constant");
  specific_gas_constant_dry = D("Physical Constants/specific gas constant dry");
  expansion_coefficient = D("Physical Constants/expansion coefficient");
  dynamic_viscosity = D("Physical Constants/dynamic viscosity");
  kinematic_viscosity = dynamic_viscosity / density;  // physical_constants.cc:150
  specific_heat_p = D("Physical Constants/specific heat p");
  specific_heat_v = D("Physical Constants/specific heat v");
  thermal_conductivity = D("Physical Constants/thermal conductivity");
  thermal_diffusivity = thermal_conductivity / (specific_heat_p * pressure);  // :156
  radiogenic_heating = D("Physical Constants/radiogenic heating");
  gravity_constant = D("Physical Constants/gravity constant");
  speed_of_sound = D("Physical Constants/speed of sound");
  atm_height = D("Physical Constants/atm height");
  R0 = D("Physical Constants/R0");
  R1 = R0 + atm_height;  // :164
}

void Parameters::parse(const PrmFile& f) {
  reference_quantities.parse(f);
  physical_constants.parse(f);
  auto S = [&](const char* p) { return f.get(p, def_of(kParameters, p)); };
  auto D = [&](const char* p) { return f.get_double(p, def_of(kParameters, p)); };
  auto I = [&](const char* p, long lo) {
    const long v = f.get_integer(p, def_of(kParameters, p));
    if (v < lo) throw PrmError(std::string("entry <") + p + "> below its pattern bound");
    return static_cast<unsigned>(v);
  };
  auto B = [&](const char* p) { return f.get_bool(p, def_of(kParameters, p)); };
  initial_global_refinement = I("Boussinesq Model/Mesh parameters/initial global refinement", 0);
  cuboid_geometry = B("Boussinesq Model/Mesh parameters/cuboid geometry");
  space_dimension = I("Boussinesq Model/space dimension", 2);
  if (space_dimension > 3) throw PrmError("space dimension must be 2 or 3");
  final_time = D("Boussinesq Model/final time");
  time_step = D("Boussinesq Model/time step");
  // boussinesq_model_parameters.cc:207 (Q12: the chained assignment also sets
  // use_FEEC_solver, which the next read overwrites).
  adapt_time_step = use_FEEC_solver = B("Boussinesq Model/adapt time step");
  nse_theta = D("Boussinesq Model/nse theta");  // Q21: parsed, unused
  nse_velocity_degree = I("Boussinesq Model/nse velocity degree", 1);
  use_FEEC_solver = B("Boussinesq Model/use FEEC solver");
  use_block_preconditioner_feec = B("Boussinesq Model/use block preconditioner feec");
  correct_pressure_to_zero_mean = B("Boussinesq Model/correct pressure to zero mean");
  use_locally_conservative_discretization =
      B("Boussinesq Model/use locally conservative discretization");
  solver_diagnostics_print_level = I("Boussinesq Model/solver diagnostics level", 0);
  use_schur_complement_solver = B("Boussinesq Model/use schur complement solver");
  use_direct_solver = B("Boussinesq Model/use direct solver");
  NSE_solver_interval = I("Boussinesq Model/NSE solver interval", 1);
  temperature_theta = D("Boussinesq Model/temperature theta");  // Q21
  temperature_degree = I("Boussinesq Model/temperature degree", 1);
  filename_output = S("Boussinesq Model/filename output");
  dirname_output = S("Boussinesq Model/dirname output");
  hello_from_cluster = B("Boussinesq Model/hello from cluster");
}

std::string Parameters::template_text() {
  // Group the declared entries by subsection, as ParameterHandler::print_parameters(Text) does.
  std::map<std::string, std::vector<std::pair<std::string, std::string>>> groups;
  auto add = [&](const Decl* b, const Decl* e) {
    for (const Decl* d = b; d != e; ++d) {
      const std::string p = d->path;
      const size_t slash = p.rfind('/');
      groups[p.substr(0, slash)].push_back({p.substr(slash + 1), d->def});
    }
  };
  add(std::begin(kParameters), std::end(kParameters));
  add(std::begin(kReferenceQuantities), std::end(kReferenceQuantities));
  add(std::begin(kPhysicalConstants), std::end(kPhysicalConstants));
  std::ostringstream out;
  out << "# Listing of Parameters\n# ---------------------\n";
  for (const auto& g : groups) {
    std::vector<std::string> subs;
    std::stringstream ss(g.first);
    std::string s;
    while (std::getline(ss, s, '/')) subs.push_back(s);
    std::string indent;
    for (const auto& name : subs) {
      out << indent << "subsection " << name << "\n";
      indent += "  ";
    }
    for (const auto& kv : g.second) out << indent << "set " << kv.first << " = " << kv.second << "\n";
    for (size_t i = subs.size(); i-- > 0;) {
      indent.resize(indent.size() - 2);
      out << indent << "end\n";
    }
    out << "\n";
  }
  return out.str();
}

Parameters Parameters::from_file(const std::string& filename) {
  std::ifstream probe(filename);
  if (!probe) {
    std::ofstream out(filename);
    out << template_text();
    throw PrmError("Input parameter file <" + filename +
                   "> not found. Creating a template file of the same name.");
  }
  Parameters p;
  p.parse(PrmFile::read(filename));
  return p;
}

double Parameters::reynolds() const {
  // core_model_data.cc:7-13
  return reference_quantities.velocity * reference_quantities.length /
         physical_constants.kinematic_viscosity;
}

double Parameters::peclet() const {
  // core_model_data.cc:16-22
  return reference_quantities.velocity * reference_quantities.length /
         physical_constants.thermal_diffusivity;
}

}  // namespace dcp
