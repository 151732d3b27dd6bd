"""setuptools entry (mirrors pyproject.toml for setuptools versions without PEP 621 support).

Build the native extensions first (``python csrc/build.py``); the wheel carries the in-tree
``.so`` files as package data."""
from setuptools import find_packages, setup

setup(
    name="ytk-learn-amd",
    version="0.2.0",
    description="MI355X-native distributed classical ML (GBDT, FM/FFM, linear, soft trees) with ytk-learn's "
                "models, configs and model formats",
    python_requires=">=3.10",
    packages=find_packages(include=["ytk_learn_amd", "ytk_learn_amd.*"]),
    package_data={"ytk_learn_amd.ops": ["*.so"], "ytk_learn_amd._native": ["*.so"]},
    install_requires=["torch>=2.4", "numpy>=1.24"],
    entry_points={"console_scripts": [
        "ytk-train = ytk_learn_amd.cli.train:main",
        "ytk-predict = ytk_learn_amd.cli.predict:main",
        "ytk-libsvm-convert = ytk_learn_amd.tools.libsvm_convert:main",
    ]},
)
