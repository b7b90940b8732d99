"""Trainer with the reference's surface (trainer.py:27-280), minus wandb and
the proprietary product-name / CSV side outputs.

  train()        one epoch: UniformSample of trainDataSize triples — on device
                 (mirec_bpr_sample) instead of the host numpy loop
                 (negative_sample.py:98-134, trainer.py:56-81) — then
                 model.OneEpoch.  config["sampler"] = "ddp_capped" uses the
                 ddp_lgcn.py variant instead (train_iterative x trainDataSize
                 candidates, at most positive_num_limit triples per positive
                 item: ddp_lgcn.py:33-35, 541-582; mirec_bpr_sample_capped).  The reference shuffles the sampled triples
                 (utils.shuffle); on-device draws are i.i.d., so the shuffle
                 is a distributional no-op and is skipped.
  test()         Recall / Precision / NDCG / HR @ topks (trainer.py:115-170)
                 through evaluate.evaluate (one propagation, HIP top-k).
  train_epoch()  test once, then epochs with a test every test_span
                 (trainer.py:237-258); best recall@topks[0] checkpoints.
"""
from __future__ import annotations

import os

import torch

from .evaluate import evaluate


class Trainer:
    def __init__(self, config: dict, dataset, model):
        self.config = config
        self.dataset = dataset
        self.model = model
        self.topks = tuple(config.get("topks", (10, 20)))
        self.seed = int(config.get("seed", 2020))
        self.epoch = 0
        self.max_recall = 0.0
        self.history = []

    def train(self):
        n = int(self.dataset.trainDataSize)
        if self.config.get("sampler", "uniform") == "ddp_capped":
            from .engine import sample_epoch_capped
            nc = int(self.config.get("train_iterative", 3)) * n
            users, pos, neg = sample_epoch_capped(self.model.graph, nc,
                                                  int(self.config.get("positive_num_limit", 3000)),
                                                  seed=self.seed, offset=self.epoch * nc)
            loss = self.model.OneEpoch(users, pos, neg)
        else:
            users, pos, neg = self.model.sample(n, seed=self.seed, offset=self.epoch * n)
            loss = self.model.OneEpoch(users, pos, neg)
            if int(self.model._sample_err.item()) != 0:
                raise RuntimeError("sampler: a user has every item as a positive")
        self.epoch += 1
        return loss

    def test(self):
        self.model.eval()
        res = evaluate(self.model, self.dataset.testDict, self.topks,
                       int(self.config.get("test_u_batch_size", 10000)))
        if res["recall"][0] > self.max_recall:
            self.max_recall = float(res["recall"][0])
            path = self.config.get("checkpoint_path")
            if path:
                self.save_model(path)
        self.model.train()
        return res

    def save_model(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save(self.model.state_dict(), path)

    def train_epoch(self, epochs: int | None = None):
        epochs = int(epochs if epochs is not None else self.config.get("epochs", 1))
        span = int(self.config.get("test_span", 10))
        self.history.append({"epoch": 0, "metrics": self.test()})
        for epoch in range(epochs):
            loss = float(self.train())
            rec = {"epoch": epoch + 1, "loss": loss}
            if epoch % span == 0:
                rec["metrics"] = self.test()
            self.history.append(rec)
        return self.history
