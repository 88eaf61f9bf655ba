"""CPU oracle for the attack hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / the timed CPU baseline. The product path
(``adversarial-attacks-on-gan-based-image-fusion_amd``) never imports it and has no CPU fallback.

Contents (plain PyTorch CPU ops, fp32 or fp64, autograd for the backward):

* ``vgg_ref``       — restates ``code/vgg.py:44-64`` (VGGBase.forward) and its positional weight
                      loading (``code/vgg.py:66-76``). **Pinned** against golden vectors produced
                      by importing the real ``code/vgg.py`` in the build container
                      (``oracle/gen_golden_vgg.py`` → ``tests/golden/vgg_*.npz``).
* ``stylegan2_ref`` — restates the rosinality StyleGAN2 synthesis the reference calls as
                      ``net.decoder`` (``code/attack/attack_main2.py:619-621``). The generator is
                      an un-vendored dependency (stylegan2-pytorch ``model.py`` + ``op/upfirdn2d``,
                      ``op/fused_act``, consumed through StyleFusion ``sf_stylegan2_hook.py`` and
                      e4e ``models/psp.py``; no version pin exists in the reference). Its published
                      algorithm is restated here. **Parity unpinned**: no reference test or fixture
                      holds generator outputs; property tests only.
* ``encoder_ref``   — the e4e ``Encoder4Editing(50, 'ir_se')`` restatement (un-vendored omertov
                      encoder4editing, no version pin: parity unpinned) and the synthetic linear
                      encoder of SURVEY.md §7 (the build's own definition).
* ``attack_ref``    — the white-box objective of ``code/attack/interpolation.py:786-818`` and the
                      torchattacks PGD update rule copied in comments at
                      ``code/attack/interpolation.py:62-96``, the Adam pixel mode of
                      ``optimize_vgg`` (``:767,822``) and the torchattacks C&W rule
                      (``:98-193``) composed with the GAN objective (torchattacks is un-vendored
                      and unpinned). The objective and the Adam mode are **pinned** to the
                      reference's own ``optimize_vgg`` executed in the build container
                      (``oracle/gen_golden_objective.py`` → ``tests/golden/objective_golden.npz``).
"""
