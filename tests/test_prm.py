"""Parameter layer (CoreModelData::Parameters / PhysicalConstants /
ReferenceQuantities restated, source/model_data/*.cc)."""
import glob
import os

import numpy as np
import pytest

import dcp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = sorted(glob.glob(os.path.join(ROOT, "configs", "*.prm")))
REF = sorted(glob.glob("/root/reference/data/*.prm"))


def test_configs_present():
    assert len(CONFIGS) >= 6


@pytest.mark.parametrize("path", CONFIGS + REF, ids=os.path.basename)
def test_parse_all(path):
    rp = dcp.load_prm(path)
    assert rp.space_dimension in (2, 3)
    assert rp.physics.time_step > 0
    assert rp.R1 > rp.R0


def test_classic_derived_quantities():
    rp = dcp.load_prm(os.path.join(ROOT, "configs", "aqua_planet_shell_test_3d-classic.prm"))
    ph = rp.physics
    # nu = mu/rho = 1e-2 -> Re = U L / nu = 100; kappa = k/(c_p p) = 1e-3 -> Pe = 1000
    assert np.isclose(1 / ph.one_over_reynolds, 100.0)
    assert np.isclose(1 / ph.one_over_peclet, 1000.0)
    assert ph.expansion_coefficient == 0.2 and ph.temperature_ref == 2.0
    assert rp.R0 == 1.0 and rp.R1 == 3.0  # R1 = R0 + atm height
    assert rp.initial_global_refinement == 2 and ph.temperature_degree == 1
    assert rp.adapt_time_step == 1 and rp.use_FEEC_solver == 0  # Q12
    assert rp.final_time == 0.09 and ph.time_step == 0.1          # Q24: one step


def test_defaults_and_errors(tmp_path):
    p = tmp_path / "minimal.prm"
    p.write_text("subsection Boussinesq Model\n  set space dimension = 3\nend\n")
    rp = dcp.load_prm(str(p))
    # declared defaults (boussinesq_model_parameters.cc:52-185, physical_constants.cc:50-131)
    assert rp.initial_global_refinement == 3
    assert rp.physics.nse_solver_interval == 1
    assert rp.physics.temperature_degree == 2
    assert np.isclose(rp.R1 - rp.R0, 1.0e5)
    assert np.isclose(rp.length, 1e4)
    bad = tmp_path / "bad.prm"
    bad.write_text("subsection Boussinesq Model\n set final time = abc\nend\n")
    with pytest.raises(dcp.DcpError):
        dcp.load_prm(str(bad))
    unbalanced = tmp_path / "unbalanced.prm"
    unbalanced.write_text("subsection Boussinesq Model\n")
    with pytest.raises(dcp.DcpError):
        dcp.load_prm(str(unbalanced))
    with pytest.raises(dcp.DcpError):
        dcp.load_prm(str(tmp_path / "missing.prm"))


def test_comments_and_unknown_entries(tmp_path):
    p = tmp_path / "c.prm"
    p.write_text("# comment\nsubsection Boussinesq Model\n  set  final   time = 2.5 # tail\n"
                 "  set unknown entry = 7\n  subsection Whatever\n    set x = 1\n  end\nend\n")
    rp = dcp.load_prm(str(p))
    assert rp.final_time == 2.5
