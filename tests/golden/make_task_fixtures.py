"""Generate tests/golden/task_embeddings.npz from the reference's task .pkl files.

The .pkl files are NEVER unpickled: `pickletools.genops` only tokenizes the opcode stream, and
we keep (a) every 4096-byte BINBYTES payload (a little-endian fp16[2048] array, dtype 'f2'/'<'
per the surrounding opcodes) and (b) every unicode string starting with "Task_" (the task
names), both in stream order. Sources (read-only, in the survey container only):
  /root/reference/neurips23_evaluation/heldout_task_with_embedding.pkl   (63 tasks)
  /root/reference/neurips23_evaluation/sample_eval_task_with_embedding.pkl (24 tasks)
Run: python tests/golden/make_task_fixtures.py
"""

import os
import pickletools

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "task_embeddings.npz")


def extract(path):
    data = open(path, "rb").read()
    embs, names = [], []
    for op, arg, _pos in pickletools.genops(data):
        if isinstance(arg, (bytes, bytearray)) and len(arg) == 4096:
            embs.append(np.frombuffer(bytes(arg), dtype="<f2").copy())
        elif op.name in ("SHORT_BINUNICODE", "BINUNICODE") and isinstance(arg, str) \
                and arg.startswith("Task_"):
            names.append(arg)
    return np.stack(embs), names


def main():
    out = {}
    for key, rel in [("heldout", "neurips23_evaluation/heldout_task_with_embedding.pkl"),
                     ("sample", "neurips23_evaluation/sample_eval_task_with_embedding.pkl")]:
        emb, names = extract(os.path.join(REF, rel))
        out[f"{key}_emb"] = emb
        out[f"{key}_names"] = np.array(names)
        print(key, emb.shape, len(names), names[:2])
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
