"""Build an experimental librgan variant with extra -D flags (GEMM tuning A/B runs).

usage: python tools/build_variant.py NAME -DFOO=1 ...   -> tools/variants/librgan_NAME.so (ships with gpurun)
(VARIANT_SRC=heads_optim.hip: the translation unit rebuilt with the flags; default conv_gemm.hip)
Run with RGAN_LIB=<that path> to load it instead of the in-tree library.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "relativisticgan_amd"))
import build as B  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    out_dir = os.path.join(ROOT, "tools", "variants")
    os.makedirs(out_dir, exist_ok=True)
    B.build()
    src = os.environ.get("VARIANT_SRC", "conv_gemm.hip")
    obj = os.path.join(out_dir, f"{src[:-4]}_{name}.o")
    subprocess.run([B.HIPCC, *B.FLAGS, *defs, "-c", os.path.join(B.CSRC, src), "-o", obj], check=True,
                   stderr=subprocess.DEVNULL)
    objs = [obj] + [os.path.join(B.BUILD, s.replace(".hip", ".o")) for s in B.SOURCES if s != src]
    so = os.path.join(out_dir, f"librgan_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", so, *objs], check=True)
    print(so)


if __name__ == "__main__":
    main()
