"""W / x-bar CSV checkpoint I/O (mpisppy/utils/wxbarutils.py, wxbarwriter.py,
wxbarreader.py), pinned to the reference's own fixture files
(mpisppy/tests/examples/w_test_data/{w_file,xbar_file}.csv, committed as
tests/golden/ref_*.csv) and asserts (mpisppy/tests/test_w_writer.py:80-113):
farmer, 3 scenarios, rho = 1, 5 PH iterations."""
import csv
import os

import numpy as np
import pytest

from helpers import REF_W, REF_XBAR, ph_options
from mpisppy_amd.examples import farmer
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.utils import wxbarutils
from mpisppy_amd.utils.wxbarreader import WXBarReader
from mpisppy_amd.utils.wxbarwriter import WXBarWriter

GOLD = os.path.join(os.path.dirname(__file__), "golden")
W_FILE = os.path.join(GOLD, "ref_w_file.csv")
XBAR_FILE = os.path.join(GOLD, "ref_xbar_file.csv")


def run(lib, device, iters, extensions=None, **extra):
    opts = ph_options(iters)
    opts.update(extra)
    ph = PH(opts, farmer.scenario_names_creator(3), farmer.scenario_creator,
            scenario_creator_kwargs={"num_scens": 3}, extensions=extensions, _native_lib=lib, _device=device)
    ph.ph_main()
    return ph


def check_writer(lib, device, tmp_path):
    wf, xf = str(tmp_path / "w.csv"), str(tmp_path / "xbar.csv")
    run(lib, device, 5, WXBarWriter, W_fname=wf, Xbar_fname=xf)
    rows = list(csv.reader(open(wf)))
    # the reference's asserts (test_w_writer.py:83-86, 92-95), places=5
    assert abs(float(rows[1][2]) - 70.84705093609978) < 5e-6
    assert abs(float(rows[3][2]) - -41.104251445950844) < 5e-6
    assert [r[:2] for r in rows] == [r[:2] for r in csv.reader(open(W_FILE))][:9]
    assert np.max(np.abs(np.array([float(r[2]) for r in rows]) - REF_W.ravel())) < 5e-6
    xr = list(csv.reader(open(xf)))
    assert abs(float(xr[1][1]) - 274.2239371483933) < 5e-6
    assert [r[0] for r in xr] == [r[0] for r in csv.reader(open(XBAR_FILE))][:3]
    assert np.max(np.abs(np.array([float(r[1]) for r in xr]) - REF_XBAR)) < 1e-6
    # append mode, as the reference (a second run adds rows)
    run(lib, device, 5, WXBarWriter, W_fname=wf, Xbar_fname=xf)
    assert len(list(csv.reader(open(wf)))) == 18 and len(list(csv.reader(open(xf)))) == 6


def check_reader(lib, device):
    ph = run(lib, device, 1, WXBarReader, init_W_fname=W_FILE, init_Xbar_fname=XBAR_FILE)
    # the reference's asserts (test_w_writer.py:97-113)
    sc = ph.local_scenarios
    assert abs(sc["scen0"]._mpisppy_model.W[("ROOT", 1)].value - 70.84705093609978) < 1e-12
    assert abs(sc["scen1"]._mpisppy_model.W[("ROOT", 0)].value - -41.104251445950844) < 1e-12
    assert abs(sc["scen0"]._mpisppy_model.xbars[("ROOT", 1)].value - 274.2239371483933) < 1e-12
    assert abs(sc["scen1"]._mpisppy_model.xbars[("ROOT", 0)].value - 96.88717449844287) < 1e-12
    assert abs(sc["scen1"]._mpisppy_model.xsqbars[("ROOT", 0)].value - 96.88717449844287 ** 2) < 1e-8
    return ph


def test_writer_matches_reference_fixture(emu, tmp_path):
    check_writer(emu, "cpu", tmp_path)


def test_reader_loads_reference_fixture(emu):
    check_reader(emu, "cpu")


def test_separate_files_round_trip(emu, tmp_path):
    ph = run(emu, "cpu", 3)
    d = str(tmp_path / "wdir")
    wxbarutils.write_W_to_file(ph, d, sep_files=True)
    assert sorted(os.listdir(d)) == ["scen0_weights.csv", "scen1_weights.csv", "scen2_weights.csv"]
    W0 = ph.W_array()
    ph._W.zero_()
    ph._bump()
    wxbarutils.set_W_from_file(d, ph, 0, sep_files=True)
    assert np.array_equal(ph.W_array(), W0)      # str(float) round-trips exactly


def test_reader_errors(emu, tmp_path):
    ph = run(emu, "cpu", 1)
    bad = tmp_path / "missing_scen.csv"
    bad.write_text("scen0,DevotedAcreage[CORN0],1.0\n")
    with pytest.raises(RuntimeError, match="could not find"):
        wxbarutils.set_W_from_file(str(bad), ph, 0)
    infeas = tmp_path / "infeasible.csv"
    infeas.write_text("".join("scen%d,%s,1.0\n" % (s, v) for s in range(3) for v in
                              ["DevotedAcreage[CORN0]", "DevotedAcreage[SUGAR_BEETS0]", "DevotedAcreage[WHEAT0]"]))
    with pytest.raises(RuntimeError, match="dual feasibility"):
        wxbarutils.set_W_from_file(str(infeas), ph, 0)
    xb = tmp_path / "xb.csv"
    xb.write_text("# comment\nDevotedAcreage[CORN0],1.0\n")
    with pytest.raises(RuntimeError, match="required variable"):
        wxbarutils.set_xbar_from_file(str(xb), ph)
