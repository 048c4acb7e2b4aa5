#!/usr/bin/env python3
"""Generate the committed golden fixtures from the Python twin (tests/golden/twin.py).

Run in the build container only:  python tests/golden/gen_golden.py
It refuses to write anything unless the twin reproduces the C1 digests recorded in SURVEY.md §8(c)
(which were computed by an independent analysis restatement).  Outputs (all small):

  golden.json   digests / counts for C1 (wc, R=10, map_n=6) and more R values, the indexer (C2),
                SipHash KATs, tokenizer KATs (inputs + expected tokens)
"""
import gzip
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import twin  # noqa: E402

# SHA-256 of mr-{r}.txt for C1 (map_n = 6, nReduce = 10)
SURVEY_C1 = {
    "mr-0.txt": "d1c35602d661e8f962a5e3adffd795e9bbaebe40776403de9baad1fd33e5e097",
    "mr-1.txt": "363443683f319575d83c9d8838151798329acbeaddfbd4609de8f72b4f67afa4",
    "mr-2.txt": "681a2a27bde7c9cc1cc3c90f0765eba1fe99d5df13984e4cccadbd66cfe95ce6",
    "mr-3.txt": "880eac12f72b7f54b6e221047e3b2e8b8914b5623e88055d5f495021b4ac8e95",
    "mr-4.txt": "0bd4c53c3ad2acef517c9f725af1cbc6c69fde46c4eab65cca727e4c17a5e572",
    "mr-5.txt": "f19630ab0876b3d67ce14fb784d273659542f45f6dbeb1910bc97e1ae5ff4b29",
    "mr-6.txt": "722de905f2b3c6c1f79c9047923ebdf281321aca6fdad76301ada946a2627ce5",
    "mr-7.txt": "d98a2881b3356e287fed11f201ba735e0b95b58fe5f38fb6635f0db447dcd7f2",
    "mr-8.txt": "6a2981400b8a5140569616d68e0ebd29d4e47afb40ac8fb2762c67d55b208589",
    "mr-9.txt": "b3983f0a960d8678f89dedc7cfb118c29f04d89727e45c69f1489f1f50d0761b",
    "final.txt": "1e49341fc47e900616d40e5de845e166eade701203d05f98843641da1bf6e64f",
    "intermediates": "fb22a2278316e4c8bb2f72ba321a995f5a001fe33cd39f3fb7780fe05442edfb",
}

# Tokenizer edge cases (wc.rs:7-10 semantics)
TOKENIZER_CASES = [
    "",
    "   \t\n  ",
    "hello world",
    "don't stop",                     # deleted ' joins fragments
    "1685-1732 and_so_on",            # '-' deleted -> 16851732, '_' is \w
    "c\u001cd e\u001ff",              # U+001C..1F are NOT White_Space: deleted, joins
    "a b\u0085c　d e",  # multi-byte White_Space splits
    "symph̸athy café",      # Mn kept
    "‘quoted’ “more” — dash",
    "zero‍width non‌joiner",  # Join_Control is \w
    "x² y½ ①",         # No (superscript / fraction / circled digit) deleted
    "- -- ... !!!",                   # tokens made only of deleted chars vanish
    "﻿bom",                      # U+FEFF (Cf) deleted
    "tab\tsep\x0bvt\x0cff\rcr",
    "ends with space ",
    "ſong Ængus ālāvātār",
    "\U0001F600smile\U0001F600",      # emoji (So) deleted
    "٠١٢ ०",      # Nd in other scripts
    "a‿b",                       # Pc (undertie) is \w
    "           |",
    " ogham math narrow",
    "x" * 40 + "-" + "y" * 40,        # long key (> 16 B), joined
    "The the THE tHe",
]

SIPHASH_KEYS = ["", "a", "the", "The", "dont", "zodiacal", "È", "café", "x" * 7, "x" * 8,
                "y" * 15, "y" * 16, "z" * 17, "0123456789abcdefghij", "ālāvātār"]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def load_corpus():
    texts = []
    for m in range(6):
        with gzip.open(os.path.join(HERE, "corpus", f"gut-{m}.txt.gz"), "rb") as f:
            texts.append(f.read().decode("utf-8"))
    return texts


def wc_digests(texts, n_reduce):
    inter, outs = twin.wc_job(texts, n_reduce)
    d = {f"mr-{r}.txt": sha(outs[r]) for r in range(n_reduce)}
    d["final.txt"] = sha(twin.final_txt(outs))
    d["intermediates"] = sha(b"".join(inter[m][r] for m in range(len(texts)) for r in range(n_reduce)))
    d["output_bytes"] = sum(len(o) for o in outs)
    d["lines"] = sum(o.count(b"\n") for o in outs)
    return d, outs


def main():
    texts = load_corpus()
    toks = [twin.tokens(t) for t in texts]
    ntok = sum(len(t) for t in toks)
    c1, outs = wc_digests(texts, 10)
    bad = [k for k, v in SURVEY_C1.items() if c1[k] != v]
    if bad:
        print("twin disagrees with SURVEY.md digests:", bad)
        return 1
    print(f"C1 digests reproduced: {ntok} tokens, {c1['lines']} lines, {c1['output_bytes']} B")

    golden = {"corpus": {"files": [f"gut-{m}.txt" for m in range(6)],
                         "bytes": [len(t.encode()) for t in texts],
                         "tokens": [len(t) for t in toks],
                         "token_stream_sha256": sha("\n".join("\n".join(t) for t in toks).encode())},
              "wc": {"10": c1}}
    for r in (1, 3, 64):
        golden["wc"][str(r)], _ = wc_digests(texts, r)
    # single-file jobs (map_n = 1)
    golden["wc_single"] = {}
    for m in range(6):
        _, o = twin.wc_job([texts[m]], 7)
        golden["wc_single"][str(m)] = {f"mr-{r}.txt": sha(o[r]) for r in range(7)}
    docs = [f"data/gut-{m}.txt" for m in range(6)]
    idx = twin.indexer_job(texts, docs, 10)
    golden["indexer"] = {"10": {f"mr-{r}.txt": sha(idx[r]) for r in range(10)}}
    golden["indexer"]["10"]["output_bytes"] = sum(len(o) for o in idx)
    golden["indexer"]["10"]["lines"] = sum(o.count(b"\n") for o in idx)
    golden["indexer"]["pairs"] = sum(len(set(t)) for t in toks)
    golden["siphash13"] = [{"key": k, "hex": (k.encode() + b"\xff").hex(),
                            "hash": f"{twin.key_hash(k):016x}"} for k in SIPHASH_KEYS]
    # SipHash-2-4 paper vectors (key 00..0f) pin the restatement's round function
    key = bytes(range(16))
    k0 = int.from_bytes(key[:8], "little")
    k1 = int.from_bytes(key[8:], "little")
    golden["siphash24_paper"] = [{"len": n, "hash": f"{twin.siphash(bytes(range(n)), 2, 4, k0, k1):016x}"}
                                 for n in (0, 1, 7, 8, 15, 63)]
    golden["tokenizer"] = [{"input": s, "tokens": twin.tokens(s)} for s in TOKENIZER_CASES]
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(golden, f, indent=1, ensure_ascii=True)
    print("wrote golden.json")
    return 0


if __name__ == "__main__":
    sys.exit(main())
