"""Train the offline byte-level BPE tokenizers used by the tests and the bench.

No Llama-3 / Qwen tokenizer is available offline, so two small byte-level BPE
tokenizers are trained on the rebuilt NQ/TriviaQA passages and given the
special tokens + chat templates of the two model families the reference
branches on (re_weighting.py:65-95):
  data/tok_llama3  <|begin_of_text|> added as BOS by the post-processor AND
                   emitted by the chat template -> the reference's double BOS;
  data/tok_qwen    ChatML template, no BOS (add_special_tokens=False path).
Deterministic (fixed corpus order, single-threaded BPE merges).
"""
import gzip
import json
import os
import sys

os.environ["RAYON_NUM_THREADS"] = "1"
os.environ["TOKENIZERS_PARALLELISM"] = "false"

from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors, trainers  # noqa: E402
from transformers import PreTrainedTokenizerFast  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
VOCAB = int(os.environ.get("CRAM_TOK_VOCAB", "8192"))

LLAMA3_TEMPLATE = (
    "{% set loop_messages = messages %}{% for message in loop_messages %}"
    "{% set content = '<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n' + message['content'] | trim"
    " + '<|eot_id|>' %}{% if loop.index0 == 0 %}{% set content = bos_token + content %}{% endif %}"
    "{{ content }}{% endfor %}{% if add_generation_prompt %}"
    "{{ '<|start_header_id|>assistant<|end_header_id|>\n\n' }}{% endif %}")
QWEN_TEMPLATE = (
    "{% for message in messages %}{% if loop.first and messages[0]['role'] != 'system' %}"
    "{{ '<|im_start|>system\nYou are a helpful assistant.<|im_end|>\n' }}{% endif %}"
    "{{'<|im_start|>' + message['role'] + '\n' + message['content'] + '<|im_end|>' + '\n'}}{% endfor %}"
    "{% if add_generation_prompt %}{{ '<|im_start|>assistant\n' }}{% endif %}")


def corpus():
    for ds in ("nq", "trivia"):
        with gzip.open(os.path.join(REPO, "data", f"{ds}_1000.json.gz"), "rt", encoding="utf-8") as f:
            for r in json.load(f):
                yield r["question"]
                yield r["wrong_answer"]
                for p in r["ori_fake"] + r["reranked_dense_ctxs"]:
                    yield p


def train(specials, vocab):
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=vocab, special_tokens=specials, show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus(), trainer=trainer)
    return tok


def main():
    l3_special = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"]
    tok = train(l3_special, VOCAB)
    bos = tok.token_to_id("<|begin_of_text|>")
    tok.post_processor = processors.TemplateProcessing(single="<|begin_of_text|> $A", pair="<|begin_of_text|> $A $B",
                                                       special_tokens=[("<|begin_of_text|>", bos)])
    fast = PreTrainedTokenizerFast(tokenizer_object=tok, bos_token="<|begin_of_text|>", eos_token="<|end_of_text|>",
                                   chat_template=LLAMA3_TEMPLATE)
    fast.save_pretrained(os.path.join(REPO, "data", "tok_llama3"))

    q_special = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]
    tokq = train(q_special, VOCAB)
    fastq = PreTrainedTokenizerFast(tokenizer_object=tokq, eos_token="<|im_end|>", pad_token="<|endoftext|>",
                                    chat_template=QWEN_TEMPLATE)
    fastq.save_pretrained(os.path.join(REPO, "data", "tok_qwen"))
    print("saved", VOCAB)


if __name__ == "__main__":
    sys.exit(main())
