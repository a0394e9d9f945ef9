"""Drop-in replacements for the reference's Re_Weighting_Strategy and Find_Best_Heads.

Same constructor / method names, argument meaning, return types and quirks as
/root/reference/utils/re_weighting.py (cited per method), with two deliberate
differences:
  * `model_name` must be a LOCAL model directory (there is no hub access); its
    name still selects the chat branch ("Llama-3" / "Qwen" substrings);
  * the dense-mask forward-pre-hooks are replaced by the "cram_hip" attention
    implementation (fused HIP kernels, O(S) bias), and cal_logits runs the
    head-batched IE sweep (cram_amd.sweep) instead of 1 + L*H full forwards.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from . import attention as _attn
from . import spans as _spans
from .bias import CredibilityBias, all_heads
from .engine import CrAMEngine
from . import sweep as _sweep


class Re_Weighting_Strategy:
    """re_weighting.py:22-138."""

    def __init__(self, model_name: str = "Llama-2-13b-chat-hf", layers_to_be_modified: dict = None,
                 bad_words_ids=None, device: str = "cuda:0"):
        # re_weighting.py:24-34
        from transformers import AutoModelForCausalLM, AutoTokenizer
        _attn.register()
        self.device = torch.device(device)
        self.tokenizer = AutoTokenizer.from_pretrained(model_name)
        self.model = AutoModelForCausalLM.from_pretrained(model_name, dtype="auto",
                                                          attn_implementation=_attn.IMPL_NAME).to(self.device)
        self.model.eval()
        self.model_name = model_name
        self.bad_words_ids = list(bad_words_ids or [])
        self.num_hidden_layers = self.model.config.num_hidden_layers
        self.model_num_attention_heads = self.model.config.num_attention_heads
        if not layers_to_be_modified:
            layers_to_be_modified = all_heads(self.num_hidden_layers, self.model_num_attention_heads)
        self.layers_to_be_modified = layers_to_be_modified
        self._engine: Optional[CrAMEngine] = None

    @property
    def engine(self) -> CrAMEngine:
        if self._engine is None:
            if not CrAMEngine.supports(self.model):
                raise NotImplementedError(f"the batched engine supports {CrAMEngine.SUPPORTED} models, not "
                                          f"{self.model.config.model_type!r}")
            self._engine = CrAMEngine.from_hf(self.model)
        return self._engine

    # ------------------------------------------------------------------ reference-semantics utility
    def edit_attention_mask(self, module, input_args: tuple, input_kwargs: dict, attention_weight: torch.Tensor,
                            head_idx: list = ()):
        """re_weighting.py:36-61: materialise the dense mask the reference hook would pass.

        Kept for API compatibility and inspection; the HIP path never builds it.
        """
        hs = input_kwargs["hidden_states"]
        dt, dev = hs.dtype, hs.device
        W = attention_weight.shape[-1]
        am = input_kwargs.get("attention_mask")
        if am is None:
            T = hs.shape[1]
            S = int(input_kwargs["position_ids"][0][-1]) + 1
            if T == 1:
                am = torch.zeros((1, 1, 1, S), dtype=dt, device=dev)
            else:
                am = torch.full((T, S), torch.finfo(dt).min, dtype=dt, device=dev).triu(1).view(1, 1, T, S)
        am = am.clone()
        if am.shape[1] == 1:
            am = am.repeat(1, self.model_num_attention_heads, 1, 1)
        vals = attention_weight.reshape(1, 1, 1, W).to(dtype=dt, device=dev)
        sel = torch.zeros((1, am.shape[1], 1, 1), dtype=torch.bool, device=dev)
        for h in head_idx:
            sel[0, h] = True
        region = am[..., :W]
        region.copy_(torch.where(sel & (region == 0), vals.expand_as(region), region))
        input_kwargs["attention_mask"] = am
        return input_args, input_kwargs

    # ------------------------------------------------------------------ prompt + weights
    def decode_with_special_attention(self, question: str = "", paras: list = (), scores: list = (),
                                      answer: str = ""):
        """re_weighting.py:63-113 -> (BatchEncoding on the device, fp16 weight [1, T])."""
        _, enc, w, _ = _spans.encode(self.tokenizer, self.model_name, question, list(paras), list(scores), answer)
        enc.pop("offset_mapping")
        return enc.to(self.device), w.to(self.device)

    def _bias(self, w16: torch.Tensor, layers_to_heads: Dict) -> CredibilityBias:
        return CredibilityBias.build([w16.reshape(1, -1).cpu()], layers_to_heads, self.num_hidden_layers,
                                     self.model_num_attention_heads, self.device, self.model.dtype)

    def _generate_kwargs(self) -> dict:
        kw = {"do_sample": False, "max_new_tokens": 100}
        if self.bad_words_ids:
            kw["bad_words_ids"] = self.bad_words_ids
        if _spans.model_family(self.model_name) == "llama3":
            kw["eos_token_id"] = [self.tokenizer.eos_token_id, self.tokenizer.convert_tokens_to_ids("<|eot_id|>")]
        return kw

    @torch.no_grad()
    def run_RAG_with_attention_weighting(self, question: str = "", paras: list = (), scores: list = ()):
        """re_weighting.py:115-138 -> (prompt, answer)."""
        model_inputs, w = self.decode_with_special_attention(question=question, paras=paras, scores=scores)
        cb = self._bias(w, self.layers_to_be_modified)
        prompt = self.tokenizer.decode(model_inputs["input_ids"][0][1:])
        with _attn.reweighting(self.model, cb):
            outputs = self.model.generate(**model_inputs, **self._generate_kwargs())
        output = self.tokenizer.decode(outputs[0][1:-1])          # drops the last id even if not EOS (:133)
        output = output[output.find(prompt) + len(prompt):]
        return prompt, output

    @torch.no_grad()
    def answer_logprobs(self, question: str = "", paras: list = (), scores: list = (), answer: str = "",
                        n_answer: Optional[int] = None) -> torch.Tensor:
        """Re-weighted teacher-forced log-probabilities of the answer tokens, fp32 [n] on the device.

        Prompt + answer is encoded as decode_with_special_attention(answer=...) does (re_weighting.py:63-113);
        one forward of the model with the credibility bias on layers_to_be_modified (the hooked forward of
        re_weighting.py:118-127) gives logits; token T-n+k is scored by log_softmax(logits[T-n-1+k]).
        n defaults to the reference's answer length convention (tokenize([answer])[0, 1:], :155).
        Not a reference method: it exposes the quantity the parity tests hold to a tolerance.
        """
        if n_answer is None:
            n_answer = int(self.tokenizer([answer], return_tensors="pt")["input_ids"].shape[1]) - 1
        model_inputs, w = self.decode_with_special_attention(question=question, paras=paras, scores=scores,
                                                             answer=answer)
        ids = model_inputs["input_ids"]
        T = ids.shape[1]
        n = max(0, min(int(n_answer), T - 1))
        if n == 0:
            return torch.zeros(0, dtype=torch.float32, device=self.device)
        cb = self._bias(w, self.layers_to_be_modified)
        with _attn.reweighting(self.model, cb):
            logits = self.model(input_ids=ids, logits_to_keep=n + 1).logits[0, :n]        # rows T-n-1 .. T-2
        lp = torch.log_softmax(logits.float(), dim=-1)
        return lp.gather(1, ids[0, T - n:].view(n, 1)).view(n)

    def _greedy_processors(self) -> float:
        """The logits processors model.generate(do_sample=False) would apply from the checkpoint's
        generation_config (re_weighting.py:127-132 passes none of its own besides bad_words_ids / eos): the
        repetition penalty is returned for the engine; any other score-changing processor raises rather than
        silently diverging from the reference's greedy ids."""
        gc = self.model.generation_config
        unsupported = {"no_repeat_ngram_size": 0, "encoder_repetition_penalty": 1.0, "min_length": 0,
                       "min_new_tokens": None, "suppress_tokens": None, "begin_suppress_tokens": None,
                       "forced_bos_token_id": None, "forced_eos_token_id": None, "sequence_bias": None,
                       "exponential_decay_length_penalty": None, "renormalize_logits": False}
        for k, default in unsupported.items():
            v = getattr(gc, k, default)
            if v not in (default, None, 0, False, [], {}):
                raise NotImplementedError(f"generation_config.{k}={v!r} is not implemented by the batched engine")
        return float(getattr(gc, "repetition_penalty", None) or 1.0)

    @torch.no_grad()
    def run_RAG_batch(self, questions: List[str], paras_list: List[list], scores_list: List[list],
                      max_new_tokens: int = 100, use_graph: bool = True) -> List[tuple]:
        """Batched greedy decode on the engine (per-row lengths and bias); same (prompt, answer) per question."""
        encs = _spans.encode_batch(self.tokenizer, self.model_name, questions, paras_list, scores_list)
        prompts = [ids.to(self.device) for ids, _, _ in encs]
        ws = [w for _, w, _ in encs]
        kw = self._generate_kwargs()
        penalty = self._greedy_processors()
        eos = kw.get("eos_token_id", self.model.generation_config.eos_token_id)
        eos = [eos] if isinstance(eos, int) else list(eos or [])
        # generate(bad_words_ids=...) as transformers applies it (NoBadWordsLogitsProcessor): a one-id sequence equal
        # to an EOS id is dropped, every other sequence (any length) is banned on the device inside the step
        bad = [list(b) for b in self.bad_words_ids if not (len(b) == 1 and b[0] in eos)]
        gens = self.engine.generate(prompts, ws, self.layers_to_be_modified, max_new_tokens=max_new_tokens,
                                    eos_ids=eos, bad_words_ids=bad, use_graph=use_graph, repetition_penalty=penalty)
        res = []
        for ids, g in zip(prompts, gens):
            full = torch.cat([ids.cpu(), torch.tensor(g, dtype=ids.dtype)])
            prompt = self.tokenizer.decode(ids[1:])
            out = self.tokenizer.decode(full[1:-1])
            res.append((prompt, out[out.find(prompt) + len(prompt):]))
        return res

    @torch.no_grad()
    def run_RAG_sharded(self, questions: List[str], paras_list: List[list], scores_list: List[list],
                        batch: int = 512, max_new_tokens: int = 100, shard_dir: Optional[str] = None,
                        group=None) -> List[tuple]:
        """(prompt, answer) of every question, each decoded exactly once across the ranks of the process group
        (RAG_test.py:64-176 loops over the dataset once): questions dealt to ranks by LPT on prompt length,
        run_RAG_batch on each rank's share in batches of at most `batch` rows, answers gathered on every rank
        (cram_amd.dist.decode_sharded); with shard_dir, answers are checkpointed per rank and a restart resumes."""
        from . import dist as _dist
        costs = [float(len(q) + sum(len(x) for x in p)) for q, p in zip(questions, paras_list)]
        keys = [_dist.unit_key(q, list(p), [float(x) for x in s]) for q, p, s in zip(questions, paras_list, scores_list)]
        run = (f"decode|{self.model_name}|{str(self.model.dtype).replace('torch.', '')}|new={int(max_new_tokens)}|"
               f"heads={_dist.unit_key(sorted((str(k), list(v)) for k, v in self.layers_to_be_modified.items()))}")

        def fn(idx):
            return [list(x) for x in self.run_RAG_batch([questions[i] for i in idx], [paras_list[i] for i in idx],
                                                        [scores_list[i] for i in idx], max_new_tokens=max_new_tokens)]
        return [tuple(a) for a in _dist.decode_sharded(fn, len(questions), costs, batch, group=group,
                                                        shard_dir=shard_dir, keys=keys, run=run)]


class Find_Best_Heads(Re_Weighting_Strategy):
    """re_weighting.py:141-175."""

    def __init__(self, model_name: str = "Llama-2-13b-chat-hf", layers_to_be_modified: list = (),
                 device: str = "cuda:0"):
        super().__init__(model_name=model_name, device=device)
        torch.manual_seed(42)
        torch.cuda.manual_seed_all(42)
        self.model_num_hidden_layers = self.model.config.num_hidden_layers
        self.model_num_attention_heads = self.model.config.num_attention_heads
        self.hidden_size = self.model.config.hidden_size

    def answer_ids(self, wrong_answer: str) -> torch.Tensor:
        """re_weighting.py:155: standalone tokenisation, first id dropped (also for tokenizers without BOS)."""
        return self.tokenizer([wrong_answer], return_tensors="pt")["input_ids"][0, 1:]

    @torch.no_grad()
    def cal_logits_tensor(self, question: str = "", paras: list = (), scores: list = (), right_answer: str = "",
                          wrong_answer: str = "my name is", round_logits: bool = False,
                          layers: Optional[List[int]] = None) -> torch.Tensor:
        """IE [L, H] (or [len(layers), H] for a subset of layers) fp32 on the device (no host sync)."""
        ans = self.answer_ids(wrong_answer)
        model_inputs, w = self.decode_with_special_attention(question=question, paras=paras, scores=scores,
                                                             answer=wrong_answer)
        layers = list(range(self.model_num_hidden_layers)) if layers is None else list(layers)
        H = self.model_num_attention_heads
        if ans.numel() == 0:   # the reference sums an empty selection: IE == 0 everywhere
            return torch.zeros((len(layers), H), dtype=torch.float32, device=self.device)
        if not CrAMEngine.supports(self.model):
            return self._ie_per_head(model_inputs["input_ids"], w, ans, round_logits, layers)
        return _sweep.ie_question(self.engine, model_inputs["input_ids"][0], w[0].cpu(), ans, layers=layers,
                                  round_logits=round_logits)

    @torch.no_grad()
    def _ie_per_head(self, ids: torch.Tensor, w16: torch.Tensor, ans: torch.Tensor,
                     round_logits: bool, layers: List[int]) -> torch.Tensor:
        """The reference algorithm itself (re_weighting.py:157-175: one un-hooked forward, then one forward per
        (layer, head) with only that head re-weighted) on the transformers model with the cram_hip kernels, for
        architectures the batched engine does not implement (GPT-2).  Answer logits in fp32 like the sweep."""
        H = self.model_num_attention_heads
        n = int(ans.numel())
        ans_d = ans.to(self.device, torch.int32)
        w_lm = self.model.get_output_embeddings().weight

        def total(cb):
            with _attn.reweighting(self.model, cb):
                hid = self.model.base_model(input_ids=ids).last_hidden_state[0, -n:]
            return self._answer_logits(hid, w_lm, ans_d, round_logits).sum()

        ori = total(None)
        out = torch.empty((len(layers), H), dtype=torch.float32, device=self.device)
        for i, l in enumerate(layers):
            for h in range(H):
                out[i, h] = ori - total(self._bias(w16, {l: [h]}))
        return out

    @staticmethod
    def _answer_logits(hidden, w_lm, ids, round_logits):
        from . import ops
        dt = hidden.dtype if hidden.dtype in ops.DTYPES else torch.bfloat16    # fp32 models (GPT-2): bf16 operands
        return ops.answer_logits(hidden.to(dt).contiguous(), w_lm.to(dt), ids, round_logits=round_logits)

    @torch.no_grad()
    def cal_logits_batch(self, questions: List[str], paras_list: List[list], scores_list: List[list],
                         wrong_answers: List[str], round_logits: bool = False, shard_dir: Optional[str] = None,
                         group=None) -> torch.Tensor:
        """IE of many questions as one device tensor [Nq, L, H] fp32 (the sweep's batched form).

        Under torch.distributed (one process per GPU) the (question, layer) units are sharded over the ranks
        (cram_amd.dist.plan: whole questions by LPT, or one question's layers snake-split when there are fewer
        questions than ranks) and assembled on every rank by one all-gather; with shard_dir every rank
        checkpoints its finished units and a restarted run resumes from them (cram_amd.dist.sweep_sharded)."""
        from . import dist as _dist
        costs = [float(len(q) + sum(len(x) for x in p) + len(a))
                 for q, p, a in zip(questions, paras_list, wrong_answers)]
        fn = lambda i, layers: self.cal_logits_tensor(questions[i], paras_list[i], scores_list[i], "",
                                                      wrong_answers[i], round_logits, layers=layers)
        keys = [_dist.unit_key(q, list(p), [float(x) for x in s], a)
                for q, p, s, a in zip(questions, paras_list, scores_list, wrong_answers)]
        run = (f"{self.model_name}|L{self.model_num_hidden_layers}|H{self.model_num_attention_heads}|"
               f"{str(self.model.dtype).replace('torch.', '')}|round_logits={bool(round_logits)}")
        return _dist.sweep_sharded(fn, len(questions), costs, self.model_num_hidden_layers,
                                   self.model_num_attention_heads, self.device, shard_dir=shard_dir, group=group,
                                   keys=keys, run=run)

    def cal_logits(self, question: str = "", paras: list = (), scores: list = (), right_answer: str = "",
                   wrong_answer: str = "my name is") -> list:
        """re_weighting.py:152-175 -> list[L][H] of Python floats (IE = ori - cur)."""
        ie = self.cal_logits_tensor(question, paras, scores, right_answer, wrong_answer)
        return ie.double().cpu().numpy().astype(np.float64).tolist()
