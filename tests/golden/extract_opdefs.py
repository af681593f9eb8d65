"""Regenerates tests/golden/wheel_opdefs.json: the REGISTER_OP input / output /
attr specs of the four ops in the reference's vendored wheel
(core/custom_op/tensorflow_nms_car_3d-0.1.0-cp36-cp36m-linux_x86_64.whl).

Static only: the wheel is opened as a zip and each op library is scanned as
bytes for its printable strings (like `strings`), nothing is loaded or run.
The op-def strings sit right after the op's name in .rodata, in registration
order (inputs, outputs, attrs).  Run in the build container (the reference is
not on the GPU box):  python tests/golden/extract_opdefs.py /root/reference
"""
import glob
import json
import os
import re
import sys
import zipfile

OPS = {"CropAndResize3D": "_crop_and_resize_3d_ops.so",
       "CropAndResize3DGradImage": "_crop_and_resize_3d_grad_image_ops.so",
       "CropAndResize3DGradBoxes": "_crop_and_resize_3d_grad_boxes_ops.so",
       "NonMaxSuppression3D": "_non_max_suppression_3d_ops.so"}
SPEC = re.compile(r"^[A-Za-z_][A-Za-z0-9_]*: ")


def strings(data, n=3):
    return [m.group().decode() for m in re.finditer(rb"[\x20-\x7e]{%d,}" % n, data)]


def main(ref):
    whl = glob.glob(os.path.join(ref, "core", "custom_op", "*.whl"))[0]
    out = {}
    with zipfile.ZipFile(whl) as z:
        for op, lib in OPS.items():
            name = [n for n in z.namelist() if n.endswith("/" + lib)][0]
            s = strings(z.read(name))
            i = s.index(op)
            specs = []
            for t in s[i + 1:]:
                if SPEC.match(t):
                    specs.append(t)
                elif specs:
                    break
            out[op] = {"library": name, "specs": specs}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wheel_opdefs.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
