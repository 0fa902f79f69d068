"""Generate ref_api_names.json: the top-level def / class names of the reference's
utils/util.py, utils/dataset.py and nets/nn.py (read as text with `ast`; nothing
from the reference is imported or executed). Run in the build container:

  python tests/golden/make_ref_api_names.py /root/reference
"""
import ast
import json
import os
import sys


def names(path):
    with open(path) as f:
        tree = ast.parse(f.read())
    return sorted(n.name for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)))


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = {m: names(os.path.join(ref, *m.split("/")) + ".py") for m in ("utils/util", "utils/dataset", "nets/nn")}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_api_names.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
