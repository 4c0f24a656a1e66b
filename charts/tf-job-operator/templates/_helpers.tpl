{{- define "tfjob.configName" -}}
{{- if .Values.config.configmap -}}{{ .Values.config.configmap }}{{- else -}}tf-job-operator-config{{- end -}}
{{- end -}}
{{- define "tfjob.hasConfig" -}}
{{- if or .Values.config.configmap (eq (.Values.cloud | default "none") "amd") -}}true{{- end -}}
{{- end -}}
