#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ from the reference's
own test data (run ONLY in the survey/build container, where the read-only
reference is mounted at /root/reference; the GPU box never runs this).

Fixtures are data: inputs and expected outputs that the reference's test
suite holds, either as files under test/data/ or as numeric array literals
inside the test specs.  Nothing here copies reference source code; the
spec files are read as text and only their number lists are kept.

Sources (all paths relative to /root/reference):
  test/data/test_cases.json                     LayerTest (test/specs/LayerTest.cpp:13)
  test/specs/LayerDeltasTest.cpp:33-125         input_x / weights / deltas / expected_output
  test/specs/BackpropagationTest.cpp:31-90       input / deltas / expected grad_w (init 1.5) / grad_b
  test/specs/ExtractLumaTest.cpp:24-28          expected luma of test/data/color_grid.png
  test/specs/SwapLumaTest.cpp:21-24            color_grid2.jpg -> color_grid2_luma_swapped.png, padding 10
  test/data/config*.json                        ConfigTest (test/specs/ConfigTest.cpp:26-45)

Images are decoded with PIL here (the reference decodes with stb_image
v2.06; PNG decode is lossless so both agree; JPEG decode can differ by a
couple of LSB -- recorded in swap_luma.json["note"]).
"""
import json
import os
import re
import shutil
import sys

REF = os.environ.get("SRCNN_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))

NUM = r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?f?"


def numbers(text):
    return [float(x.rstrip("f")) for x in re.findall(NUM, text)]


def array_literal(src, pattern):
    """Return the numbers of the brace-initialiser that follows `pattern`."""
    m = re.search(pattern, src)
    if not m:
        raise SystemExit("pattern not found: %s" % pattern)
    start = src.index("{", m.end() - 1 if src[m.end() - 1] == "{" else m.end())
    depth, i = 0, start
    while True:
        c = src[i]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                break
        i += 1
    body = src[start + 1:i]
    body = re.sub(r"//[^\n]*", "", body)          # drop line comments
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return numbers(body)


def read(p):
    with open(os.path.join(REF, p)) as fh:
        return fh.read()


def dump(name, obj):
    with open(os.path.join(OUT, name), "w") as fh:
        json.dump(obj, fh, indent=1)
    print("wrote", name)


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not mounted at %s" % REF)

    # LayerTest fixture: a data file of the reference's test suite.
    with open(os.path.join(REF, "test/data/test_cases.json")) as fh:
        cases = json.load(fh)
    dump("layer_test_cases.json", cases)

    src = read("test/specs/LayerDeltasTest.cpp")
    deltas_fx = {
        "source": "test/specs/LayerDeltasTest.cpp:33-125",
        "n_prev_layer": 2, "n_next": 3, "f_next": 3, "curr_w": 5, "curr_h": 5,
        "next_w": 3, "next_h": 3,
        "input_x": array_literal(src, r"float input_x\[INPUT_SIZE\]\s*="),
        "weights": array_literal(src, r"float weights\[WEIGHTS_SIZE\]\s*="),
        "deltas": array_literal(src, r"float deltas\[DELTAS_SIZE\]\s*="),
        "expected": array_literal(src, r"std::vector<float> expected_output\s*="),
    }
    assert len(deltas_fx["input_x"]) == 50 and len(deltas_fx["weights"]) == 54
    assert len(deltas_fx["deltas"]) == 27 and len(deltas_fx["expected"]) == 50
    dump("layer_deltas.json", deltas_fx)

    src = read("test/specs/BackpropagationTest.cpp")
    bp = {
        "source": "test/specs/BackpropagationTest.cpp:31-90",
        "n_prev": 2, "n_cur": 3, "f": 3, "in_w": 5, "in_h": 5,
        "grad_w_init": 1.5,
        "input": array_literal(src, r"float input\[INPUT_SIZE\]\s*="),
        "deltas": array_literal(src, r"float deltas\[DELTAS_SIZE\]\s*="),
        "expected_grad_w": array_literal(src, r"std::vector<float> expected_weights\s*="),
        "expected_grad_b": array_literal(src, r"std::vector<float> expected_bias\s*="),
    }
    assert len(bp["input"]) == 50 and len(bp["deltas"]) == 27
    assert len(bp["expected_grad_w"]) == 54 and len(bp["expected_grad_b"]) == 3
    dump("backprop.json", bp)

    from PIL import Image
    src = read("test/specs/ExtractLumaTest.cpp")
    img = Image.open(os.path.join(REF, "test/data/color_grid.png")).convert("RGBA")
    el = {
        "source": "test/specs/ExtractLumaTest.cpp:24-28, test/data/color_grid.png",
        "w": img.size[0], "h": img.size[1],
        "rgba": list(img.tobytes()),
        "expected_normalized": array_literal(src, r"std::vector<float> output\s*="),
    }
    assert len(el["expected_normalized"]) == el["w"] * el["h"] == 25
    dump("extract_luma.json", el)

    src_img = Image.open(os.path.join(REF, "test/data/color_grid2.jpg")).convert("RGBA")
    exp_img = Image.open(os.path.join(REF, "test/data/color_grid2_luma_swapped.png")).convert("RGBA")
    sl = {
        "source": "test/specs/SwapLumaTest.cpp:21-24, test/data/color_grid2.jpg, "
                  "test/data/color_grid2_luma_swapped.png",
        "note": "input JPEG decoded by PIL, the reference decodes with stb_image "
                "v2.06: a few channels differ by <=2 LSB, so exact parity is "
                "pinned only where both decoders agree",
        "padding": 10,
        "w": src_img.size[0], "h": src_img.size[1],
        "rgba": list(src_img.tobytes()),
        "expected_rgba": list(exp_img.tobytes()),
    }
    dump("swap_luma.json", sl)

    cfg_dir = os.path.join(OUT, "config")
    os.makedirs(cfg_dir, exist_ok=True)
    for name in ("config.json", "config_invalid_val.json", "config_non_parseable.json"):
        shutil.copyfile(os.path.join(REF, "test/data", name), os.path.join(cfg_dir, name))
        print("copied config/" + name)


if __name__ == "__main__":
    main()
