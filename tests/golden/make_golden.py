"""Generate the committed golden fixtures from the reference's own test data.

Run once, in the build container (the reference tree does not exist on the GPU box):

    python tests/golden/make_golden.py /root/reference/test/matrices.jl

Inputs: the six SuiteSparse matrices that the reference embeds as literal `sparse(I, J, V, m, n)`
text in test/matrices.jl:4-9 (generated offline by test/makematrices.jl via MatrixDepot).  We only
parse that text as data; no reference code is executed.

Outputs (tests/golden/):
  matrices.npz   per matrix <key>_I/_J/_V (1-based triplets as written), <key>_shape, <key>_sym
                 (1 when the entry is Symmetric(..., :L) and must be expanded to full, as
                 runtests.jl:18 `SparseMatrixCSC(A)` does), plus seeded random probes
                 <key>_xf / <key>_yf = A*xf and <key>_xt / <key>_yt = A'*xt computed by scipy in fp64.
  MANIFEST.json  names, shapes, nnz of the expanded matrices and the generating command.

The one-hot expected outputs of the reference protocol (runtests.jl:29-53) are the columns/rows of
A itself, so they need no separate storage.
"""
import json
import re
import sys
from pathlib import Path

import numpy as np
import scipy.sparse as sp

HERE = Path(__file__).resolve().parent

ENTRY = re.compile(
    r'"(?P<key>[^"]+)"\s*=>\s*(?P<sym>Symmetric\()?sparse\(\[(?P<I>[^\]]*)\],\s*\[(?P<J>[^\]]*)\],'
    r'\s*(?P<Vt>[A-Za-z0-9]+)?\[(?P<V>[^\]]*)\],\s*(?P<m>\d+),\s*(?P<n>\d+)\)(?:,\s*Symbol\("(?P<uplo>[UL])"\)\))?'
)


def parse(text):
    out = {}
    for mt in ENTRY.finditer(text):
        vals = [v.strip() for v in mt["V"].split(",")]
        is_int = all(re.fullmatch(r"-?\d+", v) for v in vals)
        out[mt["key"]] = dict(
            I=np.array([int(v) for v in mt["I"].split(",")], dtype=np.int64),
            J=np.array([int(v) for v in mt["J"].split(",")], dtype=np.int64),
            V=np.array([float(v) for v in vals], dtype=np.float64),
            is_int=is_int,
            eltype=mt["Vt"] or ("Int64" if is_int else "Float64"),
            m=int(mt["m"]),
            n=int(mt["n"]),
            sym=1 if mt["sym"] else 0,
            uplo=mt["uplo"] or "",
        )
    return out


def to_csc(e):
    A = sp.csc_matrix((e["V"], (e["I"] - 1, e["J"] - 1)), shape=(e["m"], e["n"]))
    if e["sym"]:
        assert e["uplo"] == "L"
        T = sp.tril(A)
        A = (T + sp.tril(T, -1).T).tocsc()
    A.sort_indices()
    return A


def main(path):
    text = Path(path).read_text()
    mats = parse(text)
    assert len(mats) == 6, sorted(mats)
    rng = np.random.default_rng(0xDEADBEEF)  # seed of runtests.jl:11
    arrays, manifest = {}, {"source": "reference test/matrices.jl:4-9", "matrices": []}
    for key, e in mats.items():
        k = key.replace("/", "__")
        A = to_csc(e)
        m, n = A.shape
        xf = rng.uniform(-1, 1, n)
        xt = rng.uniform(-1, 1, m)
        arrays[k + "_I"] = e["I"]
        arrays[k + "_J"] = e["J"]
        arrays[k + "_V"] = e["V"]
        arrays[k + "_shape"] = np.array([m, n], dtype=np.int64)
        arrays[k + "_sym"] = np.array([e["sym"]], dtype=np.int64)
        arrays[k + "_int"] = np.array([int(e["is_int"])], dtype=np.int64)
        arrays[k + "_xf"] = xf
        arrays[k + "_yf"] = A @ xf
        arrays[k + "_xt"] = xt
        arrays[k + "_yt"] = A.T @ xt
        manifest["matrices"].append(dict(key=key, file_key=k, m=m, n=n, nnz=int(A.nnz),
                                         stored=int(len(e["V"])), symmetric=bool(e["sym"]),
                                         integer_values=bool(e["is_int"]),
                                         eltype=e["eltype"]))
    np.savez_compressed(HERE / "matrices.npz", **arrays)
    manifest["command"] = "python tests/golden/make_golden.py " + str(path)
    (HERE / "MANIFEST.json").write_text(json.dumps(manifest, indent=1) + "\n")
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/test/matrices.jl")
