"""Learn the shipped byte-level BPE merges from synthetic cluster-state text.

    python tools/train_tokenizer.py [--merges 8000]

Writes k8s_llm_monitor_amd/engine/data/bpe_merges.json (committed; deterministic for a seed).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_llm_monitor_amd.engine.tokenizer import DEFAULT_MERGES, ByteBPETokenizer, train_bpe  # noqa: E402
from k8s_llm_monitor_amd.llm.synthetic import QUESTIONS, synthetic_cluster_prompt  # noqa: E402


def corpus():
    for s in range(400):
        yield synthetic_cluster_prompt(s, n_nodes=8 + s % 24, n_pods=40 + 3 * (s % 50))
    try:
        from k8s_llm_monitor_amd.llm.corpus import corpus_texts
        yield from corpus_texts()
    except ImportError:
        pass
    for q in QUESTIONS:
        yield q * 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--merges", type=int, default=8000)
    a = ap.parse_args()
    m = train_bpe(corpus(), a.merges)
    ByteBPETokenizer(m).save(DEFAULT_MERGES)
    print(f"{len(m)} merges -> {DEFAULT_MERGES}")


if __name__ == "__main__":
    main()
