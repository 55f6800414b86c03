"""CPU oracle for the 5-channel 3D U-Net training step — TEST INFRASTRUCTURE ONLY.

This package is a from-scratch CPU restatement (PyTorch CPU, fp32, NCDHW) of the
reference hot path:

* ``models/unet3d.py``  (UNet3D / DoubleConv3D / Down3D / Up3D, init and forward)
* ``utils/losses.py``   (DiceLoss, BCEDiceLoss)
* ``utils/trainer.py:179-195`` (the per-batch step: zero_grad, forward, loss,
  backward, Adam(lr, weight_decay=1e-5))

It is the *checker*, never the thing measured or shipped.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``pcms_amd``) never imports it and fails loudly when the
HIP library is missing.

Parity pin: ``tests/golden/*.npz`` were produced by importing the reference's
own ``models/unet3d.py`` and ``utils/losses.py`` in the build container
(``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py`` checks this
restatement against them.
"""
