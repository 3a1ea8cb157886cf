module github.com/noise-erasurecode-plugin-amd/infectious

go 1.21
