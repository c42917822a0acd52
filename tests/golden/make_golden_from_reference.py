"""Extract the reference's own golden step vectors into JSON fixtures.

Run HERE (the reference is mounted at /root/reference only in the build container):

    python tests/golden/make_golden_from_reference.py

The reference keeps its known-answer cases as ``@pytest.mark.parametrize`` tables in
``MADN/test.py`` (classic 7-460, deterministic 478-931) and ``DOG/test.py``
(normal 6-375, neg 391-514, swap 527-629, hot-7 642-820).  This script parses those
files with ``ast`` (nothing from the reference is imported or executed), turns every
``jnp.array(x)`` literal into plain data, and writes one JSON list per test function.
Only data (inputs and expected outputs) lands in ``tests/golden/``.
"""
import ast
import json
import os
import sys

REF = os.environ.get("MUZ_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


class _StripJnp(ast.NodeTransformer):
    # jnp.array(<literal>) / jnp.int32(<literal>) -> <literal>
    def visit_Call(self, node):
        self.generic_visit(node)
        f = node.func
        if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id == "jnp":
            return node.args[0]
        return node


def _cases(path, func_name):
    tree = ast.parse(open(path).read())
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name == func_name:
            deco = node.decorator_list[0]
            names = [s.strip() for s in ast.literal_eval(deco.args[0]).split(",")]
            table = _StripJnp().visit(deco.args[1])
            out = []
            for i, elt in enumerate(table.elts):
                vals = ast.literal_eval(elt)
                case = dict(zip(names, vals))
                case["case_id"] = i
                case["source"] = f"{os.path.relpath(path, REF)}:{elt.lineno}"
                out.append(case)
            return out
    raise KeyError(func_name)


def main():
    jobs = {
        "detmadn_step_cases.json": ("MADN/test.py", "test_normal_move_deterministic_MADN"),
        "classic_madn_step_cases.json": ("MADN/test.py", "test_normal_move_classic_MADN"),
        "dog_normal_move_cases.json": ("DOG/test.py", "test_normal_move"),
        "dog_neg_move_cases.json": ("DOG/test.py", "test_neg_move"),
        "dog_swap_move_cases.json": ("DOG/test.py", "test_swap_move"),
        "dog_hot7_move_cases.json": ("DOG/test.py", "test_7_move"),
    }
    for fname, (rel, fn) in jobs.items():
        cases = _cases(os.path.join(REF, rel), fn)
        with open(os.path.join(OUT, fname), "w") as f:
            f.write("[\n" + ",\n".join(json.dumps(c) for c in cases) + "\n]\n")
        print(f"{fname}: {len(cases)} cases from {rel}:{fn}")


if __name__ == "__main__":
    sys.exit(main())
