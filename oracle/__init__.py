"""CPU oracle for the UP-Retinex hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/.  The product path (retinex-image-enhancement_amd/) never
imports it: it is the checker, never the thing measured or shipped.

Modules
  net        functional torch-CPU fp32 restatement of models/model.py forward
  cv_u8      numpy restatement of the OpenCV 8-bit colour/CLAHE/Laplacian/Gaussian
             arithmetic that enhancers/adaptive_params.py and content_aware.py call
  enhancers  restatement of the enhancer pipelines (adaptive/CLAHE, multi-scale,
             content-aware) built on net + cv_u8

Pinning: net + the multi-scale enhancer are pinned against golden vectors
produced by the reference itself (tests/golden/make_golden.py, G1-G5, G8).
cv_u8 (OpenCV arithmetic) is "parity unpinned": cv2 is not installed in the
build container, so it is pinned only by hand-derived known-answer tests.
"""
