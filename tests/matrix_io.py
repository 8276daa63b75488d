"""Writes the reference's matrix files (Learner::SaveMatrices,
src/Learner.cpp:82-123; WriteCsrMtx src/Utils.cpp:204-214) from the oracle's
enumerated paths, and reads them back (ReadCsrMtx :184-202) -- test
infrastructure for matrix-file mode (-m)."""
import numpy as np


def _write_csr(path, rows, cols, data):
    with open(path, "w") as f:
        for r in range(len(rows) - 1):
            f.write("".join(f"{int(cols[k])} {repr(float(data[k])) if data is not None else 1} "
                            for k in range(rows[r], rows[r + 1])))
            f.write("\n")


def write_matrices(oracle, prefix):
    """prefix.{C,M,P,prob,aux} for the oracle's recognized strings"""
    prow, pcol, pdata, mrow = oracle.paths()
    n = oracle.n
    ccol = oracle.ccol()
    _write_csr(prefix + ".C", np.arange(n + 1), ccol, None)
    _write_csr(prefix + ".M", mrow, np.arange(mrow[-1]), None)
    _write_csr(prefix + ".P", prow, pcol, pdata)
    with open(prefix + ".prob", "w") as f:
        for v in oracle.p():
            f.write(repr(float(v)) + "\n")
    i = oracle.info
    with open(prefix + ".aux", "w") as f:
        for v in (i["common_support"], i["plogp"], i["model_volume"], i["aux_hessian"]):
            f.write(repr(float(v)) + "\n")
        f.write(f"{int(i['aux_params'])}\n")


def read_csr(path):
    rows, cols, data = [0], [], []
    with open(path) as f:
        for line in f:
            tok = line.split()
            for k in range(0, len(tok) - 1, 2):
                cols.append(int(tok[k]))
                data.append(float(tok[k + 1]))
            rows.append(len(cols))
    return np.array(rows), np.array(cols, dtype=np.int64), np.array(data)
