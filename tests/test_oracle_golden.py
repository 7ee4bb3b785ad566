"""Pin the CPU oracle (oracle/knn_oracle.cpp) to the reference's own outputs.

Every fixture in tests/golden/ was produced by running the compiled
reference (/root/reference/knn_mpi.cpp under mpirun, see make_golden.py).
The oracle must reproduce, bit for bit:
  * Test_label.csv                          (cpp:383-393)
  * the `accuracy = ` line                  (cpp:340-349)
  * the first K+2 sorted records per query  (idx and fp64 dis, cpp:366)
"""
import numpy as np
import pytest

import golden_io
import oracle

FIXTURES = golden_io.names()


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_reference(name, fmt_cout):
    fx = golden_io.Fixture(name)
    s = fx.spec
    tr, trl, te, tel, va, val_ = fx.normalized()
    ndump = fx.test_nbr_idx.shape[1]
    nq = fx.test_nbr_idx.shape[0]
    eu = s["Euclidean_distance"]
    # Large fixtures (the reference's MNIST-shaped default config) are checked
    # on the dumped query subset to keep the CPU suite within minutes.
    full = nq == s["N_test"]
    labels, idx, dist = oracle.knn(tr, trl, te[:nq], s["K"], eu, s["class_cnt"], n_out=ndump)
    np.testing.assert_array_equal(labels, fx.test_labels[:nq])
    np.testing.assert_array_equal(idx, fx.test_nbr_idx)
    assert (dist.view(np.int64) == fx.test_nbr_dist.view(np.int64)).all()
    if s["Validation"]:
        nv = fx.val_nbr_idx.shape[0]
        vl, vidx, vdist = oracle.knn(tr, trl, va[:nv], s["K"], eu, s["class_cnt"], n_out=ndump)
        np.testing.assert_array_equal(vidx, fx.val_nbr_idx)
        assert (vdist.view(np.int64) == fx.val_nbr_dist.view(np.int64)).all()
        if full:
            assert "accuracy = " + fmt_cout(oracle.acc(val_, vl)) == str(fx.accuracy_line)


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_inputs_regenerate(name, tmp_path):
    """The generator reproduces the exact CSV bytes the reference read."""
    fx = golden_io.Fixture(name)
    s = fx.spec
    fx.write_inputs(str(tmp_path))  # asserts the sha256 recorded by the reference run
    tr, trl, te, tel, va, val_ = fx.sets()
    # atof of the CSV text (the reference's parser) gives the generator's doubles
    data, lab, n = oracle.read_csv(str(tmp_path / "train.csv"), s["dim"], True, s["N_train"])
    np.testing.assert_array_equal(data, tr)
    np.testing.assert_array_equal(lab, trl)
    data, _, n = oracle.read_csv(str(tmp_path / "test.csv"), s["dim"], False, s["N_test"])
    np.testing.assert_array_equal(data, te)


def test_oracle_csv_reader_matches_generator(tmp_path):
    fx = golden_io.Fixture("f5_csv_crlf")   # CRLF, no trailing newline
    s = fx.spec
    tr, trl, te, tel, va, val_ = fx.write_inputs(str(tmp_path))
    data, lab, n = oracle.read_csv(str(tmp_path / "train.csv"), s["dim"], True, s["N_train"])
    assert n == s["N_train"] * (s["dim"] + 1)
    np.testing.assert_array_equal(data, tr)
    np.testing.assert_array_equal(lab, trl)
    data, _, n = oracle.read_csv(str(tmp_path / "test.csv"), s["dim"], False, s["N_test"])
    np.testing.assert_array_equal(data, te)
