"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's hot path (the oracle).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything from this package, and only as the checker / the reported CPU baseline, never as the thing
measured or shipped. The product path (``two_tower_recommender_model_amd``) never imports it and
has no CPU fallback.

Pinning: the reference (alexmillerdb/two_tower_recommender_model) is Python notebooks whose
arithmetic lives in torchrec==0.7.0 / fbgemm-gpu==0.7.0 (``requirements.txt:1-3``), neither of which
is installed or vendored here. The reference's OWN hot-path code (``transform_to_torchrec_batch``
03_model_training.py:353-382, ``TwoTower`` :395-437, ``TwoTowerTrainTask`` :440-455) is pinned by
golden vectors that ``tests/golden/make_golden.py`` produced by executing those exact functions
(extracted from the reference file at generation time) on top of this restatement. The torchrec /
fbgemm arithmetic underneath (EmbeddingBagCollection sum pooling, Perceptron, RowWiseAdagrad,
permute/bucketize) is restated from those packages' published algorithms — parity against
TorchRec itself is unpinned (no torchrec in this container, no reference test vectors for it).
"""
