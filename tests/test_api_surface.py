"""Every public name of the reference API exists in heat_amd."""
import importlib

import heat_amd as ht

groups = {
"top": "add bitwise_and bitwise_not bitwise_or bitwise_xor cumprod cumproduct cumsum diff div divide floordiv floor_divide fmod invert left_shift mod mul multiply neg negative pos positive pow power prod remainder right_shift sub subtract sum angle conj conjugate imag real e Euler inf Inf Infty Infinity nan NaN pi Device cpu get_device sanitize_device use_device exp expm1 exp2 log log2 log10 log1p logaddexp logaddexp2 sqrt square arange array asarray empty empty_like eye full full_like linspace logspace meshgrid ones ones_like zeros zeros_like nonzero where load load_csv save supports_hdf5 supports_netcdf all allclose any isclose isfinite isinf isnan isneginf isposinf logical_and logical_not logical_or logical_xor signbit balance column_stack concatenate diag diagonal dsplit expand_dims flatten flip fliplr flipud hsplit hstack moveaxis pad ravel redistribute repeat reshape resplit roll rot90 row_stack shape sort split squeeze stack swapaxes tile topk unique vsplit vstack copy sanitize_memory_layout get_printoptions set_printoptions eq equal ge greater greater_equal gt le less less_equal lt ne not_equal abs absolute ceil clip fabs floor modf round trunc sanitize_in sanitize_infinity sanitize_in_tensor sanitize_lshape sanitize_out sanitize_sequence scalar_to_1d argmax argmin average bincount cov histc histogram kurtosis max maximum mean median min minimum percentile skew std var acos acosh asin asinh atan atan2 atanh arccos arccosh arcsin arcsinh arctan arctan2 arctanh cos cosh deg2rad degrees rad2deg radians sin sinh tan tanh datatype number integer signedinteger unsignedinteger bool bool_ floating int8 byte int16 short int32 int int64 long uint8 ubyte float32 float float_ float64 double flexible can_cast canonical_heat_type heat_type_is_exact heat_type_is_inexact iscomplex isreal issubdtype heat_type_of promote_types result_type complex64 cfloat csingle complex128 cdouble finfo iinfo MPI MPI_WORLD MPI_SELF CUDA_AWARE_MPI MPIRequest Communication MPICommunication get_comm sanitize_comm use_comm BaseEstimator ClassificationMixin ClusteringMixin RegressionMixin is_classifier is_clusterer is_estimator is_regressor DNDarray dot matmul matrix_norm norm outer projection trace transpose tril triu vecdot vector_norm qr cg lanczos",
"linalg": "dot matmul matrix_norm norm outer projection trace transpose tril triu vecdot vector_norm qr cg lanczos",
"random": "get_state normal permutation rand ranf randint random_integer randn random random_sample randperm sample seed set_state standard_normal",
"tiling": "SplitTiles SquareDiagTiles",
"spatial": "cdist manhattan rbf",
"cluster": "KMeans KMedians KMedoids Spectral",
"graph": "Laplacian", "regression": "Lasso", "naive_bayes": "GaussianNB", "classification": "KNeighborsClassifier",
"nn": "DataParallel DataParallelMultiGPU functional Linear Conv2d ReLU MSELoss Module Sequential",
"optim": "DataParallelOptimizer DASO utils lr_scheduler SGD Adam",
"utils.data": "DataLoader Dataset dataset_shuffle dataset_ishuffle dataset_irecv PartialH5Dataset PartialH5DataLoaderIter MNISTDataset matrixgallery",
"utils": "vision_transforms",
}
def test_public_api_surface():
    missing = []
    for g, names in groups.items():
        mod = ht if g == "top" else ht.linalg if g == "linalg" else ht.random if g == "random" else ht.tiling if g == "tiling" else importlib.import_module("heat_amd." + g)
        for n in names.split():
            if not hasattr(mod, n):
                missing.append(g + "." + n)
    meth = "T abs absolute acos all allclose any argmax argmin asin atan atan2 average balance ceil clip copy cos cosh exp exp2 expand_dims expm1 fabs flatten floor isclose kurtosis log log10 log1p log2 max mean median min modf nonzero norm prod qr redistribute reshape resplit rot90 round save sin sinh skew sqrt square squeeze std sum swapaxes tan tanh trace transpose tril triu trunc unique var __matmul__ __add__ __radd__ __and__ __or__ __xor__ __lshift__ __rshift__ __invert__ __neg__ __pos__ __pow__ __rpow__ __mod__ __floordiv__ __truediv__ __rtruediv__ __eq__ __ne__ __lt__ __le__ __gt__ __ge__ __abs__ __len__ __iter__ __float__ __int__ __bool__ __complex__ get_halo array_with_halos astype balance_ counts_displs create_lshape_map fill_diagonal is_balanced is_distributed numpy redistribute_ resplit_ lshape_map halo_next halo_prev larray gshape lshape split device comm dtype ndim size gnumel lnumel nbytes gnbytes lnbytes imag real shape stride strides balanced tolist item __setitem__ __getitem__ __str__ __repr__ __torch_proxy__ __array__ cpu".split()
    x = ht.zeros((3,3))
    for m in meth:
        if not hasattr(x, m):
            missing.append("DNDarray." + m)
    assert not missing, missing
