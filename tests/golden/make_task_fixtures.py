"""Generate tests/golden/task_embeddings.npz from the reference's task .pkl files.

The .pkl files are NEVER unpickled: `pickletools.genops` only tokenizes the opcode stream, and
we keep (a) every 4096-byte BINBYTES payload (a little-endian fp16[2048] array, dtype 'f2'/'<'
per the surrounding opcodes), (b) every unicode string starting with "Task_" (the task
names), both in stream order, and (c) each TaskSpec's (eval_fn, eval_fn_kwargs, sampling_weight)
read off the opcode stream: strings, ints and floats as the opcodes carry them, memo gets
resolved to the value that was memoized, and a class reference (STACK_GLOBAL of a module and a
name string) to its name — a tokenizer's bookkeeping, nothing is constructed or called. Sources (read-only, in the survey container only):
  /root/reference/neurips23_evaluation/heldout_task_with_embedding.pkl   (63 tasks)
  /root/reference/neurips23_evaluation/sample_eval_task_with_embedding.pkl (24 tasks)
Run: python tests/golden/make_task_fixtures.py
"""

import json
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


def extract_specs(path):
    """[(eval_fn, kwargs, sampling_weight)] of every TaskSpec in the pickle's opcode stream."""
    data = open(path, "rb").read()
    memo, toks, strs, last = {}, [], [], None
    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("SHORT_BINUNICODE", "BINUNICODE", "UNICODE"):
            last = arg
            toks.append(arg)
            strs.append(arg)
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "INT", "BINFLOAT", "FLOAT"):
            last = arg
            toks.append(arg)
        elif n == "MEMOIZE":
            memo[len(memo)] = last
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = last
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            last = memo.get(arg)
            toks.append(last)
        elif n == "STACK_GLOBAL":  # module, name -> a marker for the class named `name`
            last = ("class", strs[-1])
            toks.append(last)
        else:
            last = None

    def is_cls(t):
        return isinstance(t, tuple) and t[0] == "class"

    specs, i = [], 0
    while i < len(toks):
        if toks[i] == "eval_fn":
            j = i + 1
            while not is_cls(toks[j]):
                j += 1
            fn = toks[j][1]
            assert toks[j + 1] == "eval_fn_kwargs"
            k, kw = j + 2, {}
            while toks[k] != "task_cls":
                key, k = toks[k], k + 1
                if isinstance(toks[k], str) and "." in toks[k] and is_cls(toks[k + 2]):
                    k += 2  # module string, name string, then the class marker
                val = toks[k]
                kw[key] = val[1] if is_cls(val) else val
                k += 1
            m = k
            while toks[m] != "sampling_weight":
                m += 1
            specs.append([fn, kw, toks[m + 1]])
            i = m
        i += 1
    return specs


def main():
    out = {}
    for key, rel in [("heldout", "neurips23_evaluation/heldout_task_with_embedding.pkl"),
                     ("sample", "neurips23_evaluation/sample_eval_task_with_embedding.pkl")]:
        emb, names = extract(os.path.join(REF, rel))
        out[f"{key}_emb"] = emb
        out[f"{key}_names"] = np.array(names)
        out[f"{key}_specs"] = np.array(json.dumps(extract_specs(os.path.join(REF, rel))))
        print(key, emb.shape, len(names), names[:2])
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
