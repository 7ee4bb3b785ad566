"""Load golden fixtures (tests/golden/*.npz) and regenerate their inputs.

Fixtures are plain arrays (np.load with allow_pickle=False).  Inputs are
regenerated from the stored generator spec and must hash to the stored
sha256, which proves the regenerated CSV bytes are the ones the reference
read when the fixture was made.
"""
import glob
import json
import os

import numpy as np

import datagen

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


class Fixture:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.arrays = {k: z[k] for k in z.files}
        self.spec = json.loads(str(self.arrays["spec"]))
        self._sets = None

    def __getattr__(self, k):
        a = self.__dict__.get("arrays", {})
        if k in a:
            return a[k]
        raise AttributeError(k)

    def write_inputs(self, d, names=("train.csv", "validation.csv", "test.csv")):
        s = self.spec
        sets, sha = datagen.write_csvs(d, s, names=names, crlf=s["crlf"],
                                       trailing_newline=s["trailing_newline"])
        assert sha == str(self.arrays["csv_sha256"]), "regenerated inputs differ"
        return sets

    def sets(self):
        """(train, train_lab, test, test_lab, val, val_lab), raw (unnormalised).
        Taken straight from the generator: its values are exact binary
        fractions printed with round-trip precision, so they equal what atof
        reads back from the CSV (test_fixture_inputs_regenerate checks the
        CSV bytes against the hash the reference run recorded)."""
        if self._sets is None:
            s = self.spec
            self._sets = datagen.make_sets(s["kind"], s["seed"], s["N_train"], s["N_test"],
                                           s["N_val"], s["dim"], s["class_cnt"])
        return self._sets

    def normalized(self):
        """Inputs after the reference's normalisation (via the oracle)."""
        import oracle
        tr, trl, te, tel, va, val_ = [a.copy() for a in self.sets()]
        s = self.spec
        if s["Normalize"]:
            oracle.normalize(tr, te, va if s["Validation"] else None)
        return tr, trl, te, tel, va, val_
