"""CPU oracle for the STF-Unet training hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``stf-unet_amd/``) imports
this package.  It may be imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` -- always as the checker, never
as the thing measured or shipped.

What it is: a plain-PyTorch fp32 CPU restatement of the reference's hot path,
written functionally (explicit parameter dicts keyed by the reference's
``state_dict`` names) so every step can be read against the reference:

* ``oracle.unet``     -- ``src/unet.py:5-57``
* ``oracle.stf``      -- ``src/stf_lstm_unet.py:7-256`` (+ a ResNet-34
                         restatement for ``torchvision.models.resnet34``)
* ``oracle.loss``     -- ``train_utils/train_and_eval.py:299-313`` and
                         ``train_utils/dice_coefficient_loss.py:5-55``
* ``oracle.metrics``  -- ``train_utils/train_and_eval.py:25-142``
* ``oracle.optim``    -- ``torch.optim.AdamW`` as configured at ``train.py:230-237``
                         and ``create_lr_scheduler`` (``train_and_eval.py:414-438``)
* ``oracle.init``     -- canonical counter-based (splitmix64) weights so that
                         full-width models need no committed weights.

Pinning: ``tests/golden/make_golden.py`` imports the reference modules by path
(in the build container only) and writes the fixtures under ``tests/golden``;
``tests/test_oracle_golden.py`` checks this restatement against them.
ResNet-34 arithmetic comes from torchvision (unpinned, absent here); the
fixtures were generated with a standard BasicBlock ResNet-34 stand-in, so the
ResNet part is pinned to the *standard* architecture, not to a torchvision
build ("parity unpinned" w.r.t. real torchvision).
"""
