"""Build an experimental librgan variant for same-box A/B runs (tools/ab_lib.sh).

usage: python tools/build_variant.py NAME [--patch FILE.diff ...] [-DFOO=1 ...]
    -> tools/variants/librgan_NAME.so (ships with gpurun; load it with RGAN_LIB=<path>)

The product sources carry no experiment switches: a variant is a patch (``git diff`` of
``relativisticgan_amd/csrc``, applied with ``patch -p1`` to a scratch copy of the tree) and/or
extra -D flags.  Every translation unit the patch touches (and, with -D flags only,
VARIANT_SRC, default conv_gemm.hip) is recompiled; the others come from the in-tree build.
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "relativisticgan_amd"))
import build as B  # noqa: E402


def main():
    name, rest = sys.argv[1], sys.argv[2:]
    patches, defs = [], []
    while rest:
        a = rest.pop(0)
        if a == "--patch":
            patches.append(os.path.abspath(rest.pop(0)))
        else:
            defs.append(a)
    out_dir = os.path.join(ROOT, "tools", "variants")
    os.makedirs(out_dir, exist_ok=True)
    scratch = tempfile.mkdtemp(prefix="rgan_variant_")
    try:
        shutil.copytree(os.path.join(ROOT, "relativisticgan_amd", "csrc"),
                        os.path.join(scratch, "relativisticgan_amd", "csrc"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(scratch, "include"))
        touched = set()
        for pf in patches:
            subprocess.run(["patch", "-p1", "-s", "-i", pf], cwd=scratch, check=True)
            for line in open(pf):
                if line.startswith("+++ ") and line.rstrip().endswith(".hip"):
                    touched.add(os.path.basename(line.split()[1]))
        if not touched:
            touched.add(os.environ.get("VARIANT_SRC", "conv_gemm.hip"))
        # the untouched translation units come from the in-tree build (built here only if
        # missing: the in-tree library may be on its way to a GPU box and is left alone)
        if any(not os.path.exists(os.path.join(B.BUILD, s.replace(".hip", ".o"))) for s in B.SOURCES if s not in touched):
            B.build()
        csrc = os.path.join(scratch, "relativisticgan_amd", "csrc")
        flags = [f if not f.startswith("-I") else "-I" + os.path.join(scratch, "include") for f in B.FLAGS]
        objs = []
        for src in B.SOURCES:
            if src in touched:
                obj = os.path.join(out_dir, f"{src[:-4]}_{name}.o")
                subprocess.run([B.HIPCC, *flags, *defs, "-c", os.path.join(csrc, src), "-o", obj], check=True)
                objs.append(obj)
            else:
                objs.append(os.path.join(B.BUILD, src.replace(".hip", ".o")))
        so = os.path.join(out_dir, f"librgan_{name}.so")
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", so, *objs], check=True)
        print(so)
    finally:
        shutil.rmtree(scratch, ignore_errors=True)


if __name__ == "__main__":
    main()
