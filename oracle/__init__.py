"""CPU oracle for the MI355X fusion hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``multimodalemotionrecognition_amd`` imports
this package; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker / the timed CPU baseline.

The oracle is a plain fp32 PyTorch-on-CPU restatement of the reference's
algorithm (Wionerlol/MultimodalEmotionRecognition @ 2026-04-17):

* ``fusion_ref``  -- ``src/models/fusion.py`` + ``src/models/temporal.py``
* ``resnet18_ref`` -- torchvision ``resnet18`` trunk as wrapped by
  ``src/models/video.py:21-23`` (torchvision 0.25.0 is not installed here, so
  this piece is **parity unpinned**)
* ``wavlm_ref``   -- transformers ``WavLMModel`` as wrapped by
  ``src/models/wavlm_audio.py:165-183``
* ``train_ref``   -- ``src/train.py:200-228`` (loss, backward, Adam)

Pinning: ``tests/test_oracle_golden.py`` checks every restated function against
golden vectors produced by importing the reference itself in the build
container (``tools/gen_golden.py`` -> ``tests/golden/*.npz``).
"""
