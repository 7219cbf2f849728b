"""Generate golden fixtures from the reference where it is importable in this container.

Only pupperv3_mjx/obstacles.py imports without jax/mujoco (stdlib only); it is
loaded by file path from /root/reference and run with the reference test fixture's
arguments (test_environment.py:29-44) to record the box attributes it writes.  Run here
(not on the GPU box): python tests/golden/make_golden.py
"""
import importlib.util
import json
import os
import xml.etree.ElementTree as ET

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    spec = importlib.util.spec_from_file_location("ref_obstacles", os.path.join(REF, "pupperv3_mjx", "obstacles.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    xml = open(os.path.join(REF, "test", "test_pupper_model.xml")).read()
    out = {}
    for seed, n, length in ((0, 10, 6.0), (3, 25, 3.0)):
        tree = ET.ElementTree(ET.fromstring(xml))
        tree = mod.add_boxes_to_model(tree, n_boxes=n, x_range=(-5, 5), y_range=(-5, 5), height=0.02,
                                      length=length, seed=seed)
        boxes = [dict(g.attrib) for g in tree.getroot().find("worldbody").findall("geom")
                 if g.get("name", "").startswith("box_geom_")]
        out[f"seed{seed}_n{n}_len{length}"] = boxes
    with open(os.path.join(HERE, "obstacles_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(out), "cases")


if __name__ == "__main__":
    main()
