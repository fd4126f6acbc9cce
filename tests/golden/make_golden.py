"""Generate the committed golden fixtures (run in the build container):

    python tests/golden/make_golden.py

* notebooks.json -- the reference's PUBLISHED example outputs, transcribed
  from examples/multivariate_normal/mvn_example.ipynb:3647-3668 and
  examples/gaussian_mixture_model/gmm_example.ipynb:6375-6416 (printed to 6
  significant digits; the notebooks print the d x n matrix transposed).
  These pin the oracle (tests/test_oracle.py).
* test_svgd_n10.json -- the tests/test_svgd.cpp:65-203 scenario run by the
  oracle (the reference test only compares its SVGD class with its own
  manual loop, it stores no numbers).
* phi_*.npz -- one-step inputs (X, G, a) and oracle outputs (phi, median,
  scale) on synthetic configurations, for the GPU parity tests.

Only the oracle (oracle/) is used; the reference is C++ with Eigen/CppAD
dependencies that are absent here, so nothing of it is executed.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as o  # noqa: E402

MVN_INIT = [[2.04113, -0.633702], [1.6986, 1.79064], [2.46988, -1.81469], [-0.988663, 1.60938],
            [-1.33335, 0.32382], [-0.135618, 0.773226], [-0.811293, 0.0804055], [2.71338, 2.49717],
            [0.81427, 1.30378], [-2.15038, 0.641813]]
MVN_FINAL = [[0.469815, 1.16686], [-0.184629, 1.82829], [0.0827075, -0.375293], [-1.04192, 2.64404],
             [-0.946601, -0.148336], [-1.73173, 1.15547], [-1.14872, -1.79038], [0.452507, 3.21318],
             [-0.791678, 0.828686], [-2.05712, -0.556122]]
GMM_INIT = [[5.443, -1.68987], [4.52959, 4.77504], [6.58636, -4.83918], [-2.63644, 4.29167],
            [-3.5556, 0.863519], [-0.361647, 2.06193], [-2.16345, 0.214415], [7.23568, 6.65912],
            [2.17139, 3.47675], [-5.73436, 1.7115], [-7.73919, -4.11381], [-5.80429, 4.86683],
            [-5.49313, -1.58489], [-5.92335, -6.25906], [7.98279, -4.50789], [0.206918, 5.4258],
            [1.80224, -3.26349], [2.20084, 0.388595], [-0.102672, 7.5644], [-3.31973, 4.34172]]
GMM_FINAL = [[3.72827, -2.73105], [0.0615133, 2.94274], [3.73122, -2.72353], [-5.18645, 3.69024],
             [-2.22385, 4.03994], [-3.70641, 6.20652], [-1.70512, 3.57094], [4.62788, 0.40819],
             [-0.490985, 4.97395], [-3.89137, 4.12686], [1.38888, -4.0669], [-6.25797, 5.65887],
             [-2.64295, 2.56246], [2.75646, -5.90763], [6.02122, -1.5987], [-2.62781, 4.86152],
             [4.93368, -4.37164], [2.36409, -1.42065], [-2.90504, 4.69648], [-4.34614, 4.82727]]


def notebooks():
    return {
        "mvn": {
            "source": "examples/multivariate_normal/mvn_example.ipynb:3647-3668; "
                      "examples/multivariate_normal/mvn_example.cpp:9-39",
            "n": 10, "d": 2, "iters": 1000, "init_scale": 3.0, "seed": 1,
            "optimizer": {"kind": "adagrad", "lr": 0.1},
            "means": [[-0.6871, 0.8010]],
            "covs": [(5 * np.array([[0.2260, 0.1652], [0.1652, 0.6779]])).tolist()],
            "initial": MVN_INIT, "final": MVN_FINAL,
        },
        "gmm": {
            "source": "examples/gaussian_mixture_model/gmm_example.ipynb:6375-6416; "
                      "examples/gaussian_mixture_model/gmm_example.cpp:9-49",
            "n": 20, "d": 2, "iters": 1000, "init_scale": 8.0, "seed": 1,
            "optimizer": {"kind": "adam", "lr": 0.1, "beta1": 0.9, "beta2": 0.999},
            "means": [[3.6871, -2.801], [-2.9802, 4.3387]],
            "covs": [(5 * np.array([[0.5001, 0.2426], [0.2426, 0.8420]])).tolist(),
                     (5 * np.array([[0.6779, -0.1652], [-0.1652, 0.2260]])).tolist()],
            "initial": GMM_INIT, "final": GMM_FINAL,
        },
    }


def test_svgd_model_grad(X):
    """∇ log(7.5 cos x0 + 10 cos x1 + 3 x0 x1 - 6) (tests/test_svgd.cpp:78-93,171-182)."""
    f = 7.5 * np.cos(X[:, 0]) + 10 * np.cos(X[:, 1]) + 3 * X[:, 0] * X[:, 1] - 6
    g = np.stack([-7.5 * np.sin(X[:, 0]) + 3 * X[:, 1], -10 * np.sin(X[:, 1]) + 3 * X[:, 0]], 1)
    return g / f[:, None]


def test_svgd_scenario():
    X0 = o.eigen_random(2, 10, 1.0, 1)
    X = o.run_svgd(X0, test_svgd_model_grad, 15, o.Adam((10, 2), 0.1, 0.9, 0.999), scale=1.0,
                   lower=np.array([-1.0, -1.0]), upper=np.array([1.0, 1.0]))
    return {"source": "tests/test_svgd.cpp:65-203 (oracle run)", "n": 10, "d": 2, "iters": 15,
            "scale": 1.0, "lower": [-1.0, -1.0], "upper": [1.0, 1.0],
            "optimizer": {"kind": "adam", "lr": 0.1, "beta1": 0.9, "beta2": 0.999},
            "initial": X0.tolist(), "final": X.tolist()}


def gmm_params(d, k, seed=0x5EED):
    mus = o.splitmix((k, d), 3.0, seed)
    covs = np.stack([np.eye(d) * (1.0 + 0.25 * c) for c in range(k)])
    return mus, covs


def phi_case(name, n, d, k, seed):
    X = o.splitmix((n, d), 3.0, seed)
    mus, covs = gmm_params(d, k, seed + 1)
    G = o.logp_grad_gmm(X, mus, covs)
    a, med = o.median_scale(X)
    ph = o.phi(X, G, a)
    np.savez(os.path.join(HERE, f"phi_{name}.npz"), X=X, G=G, a=a, med=med, phi=ph, mus=mus, covs=covs)


def main():
    with open(os.path.join(HERE, "notebooks.json"), "w") as f:
        json.dump(notebooks(), f, indent=1)
    with open(os.path.join(HERE, "test_svgd_n10.json"), "w") as f:
        json.dump(test_svgd_scenario(), f, indent=1)
    phi_case("n256_d2", 256, 2, 1, 11)
    phi_case("n1000_d8", 1000, 8, 4, 12)
    phi_case("n300_d64", 300, 64, 1, 13)
    phi_case("n77_d3", 77, 3, 2, 14)


if __name__ == "__main__":
    main()
