k_learnable_affine_parameters = True  # deeplab/config.py:1 of the reference
