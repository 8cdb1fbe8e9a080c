"""owl_wms.nn on libowlk: the reference's module API (owl_wms/nn) with HIP kernels underneath."""
