"""Extract the recorded is_soft_locked / dice_probabilities outputs of the reference notebook into a fixture.

Run HERE (the reference is mounted at /root/reference only in the build container):

    python tests/golden/make_dice_golden_from_notebook.py

``MADN/jupyter_code/test_functions.ipynb`` cells 3-4 set up eight 2-player classic-MADN positions
(``env_reset(0, num_players=2, distance=10, enable_dice_rethrow=..., enable_start_on_1=...)``, pins set by
hand, board = set_pins_on_board) and hold the printed outputs of ``is_soft_locked`` and
``dice_probabilities`` (MADN/classic_madn.py:180-228) for each.  The notebook is read as JSON; the rule flags
and pin arrays are read from the cell text with regular expressions and the outputs from the recorded
stdout.  Nothing from the reference is imported or executed; only data lands in tests/golden/.

Board layout: the notebook's outputs were recorded with an older classic_madn.py whose track had
num_players x distance cells (cell 1's printed 2-player board is 2 rows of 10), so its goal cells started at
20 for 2 players: pins 23 / 22 are player 0's goal slots 3 / 2 there.  The current code has 4 x distance = 40
track cells and goal slots at 40 + 4 * seat + j (classic_madn.py:74-89).  Each case keeps the notebook's pins
as ``pins_notebook`` and the same placement in today's layout as ``pins`` (track cells unchanged, a goal cell
20 + 4 s + j -> 40 + 4 s + j).
"""
import json
import os
import re

REF = os.environ.get("MUZ_REFERENCE", "/root/reference")
NB = os.path.join(REF, "MADN", "jupyter_code", "test_functions.ipynb")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "classic_dice_notebook_cases.json")

_RESET = re.compile(r"env_reset\(0,\s*num_players=(\d+),\s*distance=(\d+),\s*enable_dice_rethrow=(True|False),"
                    r"\s*enable_start_on_1=(True|False)\)")
_PINS = re.compile(r"env\.pins = jnp\.array\((\[\[.*?\]\])", re.S)
_SOFT = re.compile(r"Soft locked:\s+(True|False)")
_PROBS = re.compile(r"Dice probabilities:\s+\[([^\]]*)\]")


def main():
    nb = json.load(open(NB))
    cases = []
    for cell_no in (3, 4):
        cell = nb["cells"][cell_no]
        src = "".join(cell["source"])
        text = "".join("".join(o.get("text", [])) for o in cell.get("outputs", []))
        resets, pins = _RESET.findall(src), _PINS.findall(src)
        softs, probs = _SOFT.findall(text), _PROBS.findall(text)
        if not (len(resets) == len(pins) == len(softs) == len(probs) == 4):
            raise SystemExit(f"cell {cell_no}: unexpected layout {len(resets)} {len(pins)} {len(softs)} {len(probs)}")
        for (P, d, rethrow, on1), pin_txt, soft, prob in zip(resets, pins, softs, probs):
            old = json.loads(re.sub(r"\s+", "", pin_txt))
            old_track = int(P) * int(d)
            new = [[x if x < old_track else 4 * int(d) + (x - old_track) for x in row] for row in old]
            cases.append({"source": f"MADN/jupyter_code/test_functions.ipynb cell {cell_no}",
                          "num_players": int(P), "distance": int(d),
                          "rules": {"enable_dice_rethrow": rethrow == "True", "enable_start_on_1": on1 == "True"},
                          "pins_notebook": old, "pins": new, "current_player": 0,
                          "soft_locked": soft == "True", "dice_probabilities": [float(x) for x in prob.split()]})
    json.dump(cases, open(OUT, "w"), indent=1)
    print(f"{len(cases)} cases -> {OUT}")


if __name__ == "__main__":
    main()
